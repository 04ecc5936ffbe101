"""Static checks of the SHA-256 kernels' machine code (csrc/sha256.hip),
compiled to assembly here (hipcc cross-compiles without a GPU).

1. The pair-lane latency kernel (sha256_chain2).  gfx9 needs two wait states
   between a VALU instruction that writes a VGPR and a DPP instruction that
   reads that VGPR through its lane permutation (the first source operand);
   the kernel's DPP adds sit inside asm statements the compiler does not look
   into, so nothing but the instruction order keeps that rule.  Every
   instruction of every sha256_chain2 instantiation is walked: for each *_dpp
   instruction, the register it permutes must not have been written by a VALU
   instruction fewer than two wait states earlier (an instruction is one wait
   state, s_nop N is N + 1).  A round must stay ten instructions.
2. Every kernel's resources as the compiler reports them: no scratch, and the
   VGPR counts the persistent kernels' launch geometry assumes."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "distributed-file-storage_amd", "csrc", "sha256.hip")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


def vregs(tok):
    """Registers named by one operand: v7 -> {7}; v[4:7] -> {4, 5, 6, 7}."""
    m = re.fullmatch(r"v(\d+)", tok)
    if m:
        return {int(m.group(1))}
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    return set()


def instructions(asm, name):
    """(mnemonic, operands) of every instruction of the kernels whose symbol
    contains `name`, in program order."""
    out, on = [], False
    for line in asm.splitlines():
        if re.match(r"^[_A-Za-z0-9]+:", line):
            on = name in line
            if on:
                out.append([])
            continue
        if not on:
            continue
        t = line.split(";")[0].strip()
        if not t or t.startswith(".") or t.endswith(":"):
            continue
        parts = t.split(None, 1)
        ops = [o.strip() for o in re.split(r",\s*(?![^\[]*\])", parts[1])] if len(parts) > 1 else []
        out[-1].append((parts[0], ops))
        if parts[0] == "s_endpgm":
            on = False
    return [k for k in out if k]


def compile_device(src, out):
    """Device code of one source file as assembly; returns (assembly text, the
    compiler's per-kernel resource remarks)."""
    cmd = [HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "-Xclang", "-target-feature", "-Xclang",
           "-packed-fp32-ops", "--cuda-device-only", "-S", "-Rpass-analysis=kernel-resource-usage", "-x", "hip", src,
           "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    return out.read_text(), r.stderr


@pytest.fixture(scope="module")
def sha_build(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("no hipcc")
    return compile_device(SRC, tmp_path_factory.mktemp("isa") / "sha256.s")


@pytest.fixture(scope="module")
def device_asm(sha_build):
    return sha_build[0]


def resources(remarks):
    """{kernel symbol: {"VGPRs": n, "VGPRs Spill": n, "ScratchSize": n, "Occupancy": n, ...}} from
    -Rpass-analysis=kernel-resource-usage."""
    out, cur = {}, None
    for line in remarks.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = out.setdefault(m.group(1), {})
            continue
        m = re.search(r"remark:\s+([A-Za-z][A-Za-z ]*?)(?: \[[^\]]*\])?: (\d+) \[-Rpass", line)
        if m and cur is not None:
            cur[m.group(1)] = int(m.group(2))
    return out


def test_sha_kernels_fit_their_wave_budgets(sha_build):
    """No kernel of sha256.hip spills to scratch, and the persistent kernels
    keep the VGPR counts their launch geometry assumes: four waves per SIMD for
    the hash-only and one-pass instantiations (<= 128 VGPRs), three for the
    fused-Base64 one (<= 168)."""
    res = resources(sha_build[1])
    kernels = {k: v for k, v in res.items() if "sha256_" in k or "static_prep" in k}
    assert len(kernels) >= 9, sorted(res)
    for k, v in kernels.items():
        assert v["ScratchSize"] == 0 and v["VGPRs Spill"] == 0 and v["VGPRs"] > 0, (k, v)
    def one(sub):
        (k,) = [k for k in kernels if sub in k]
        return kernels[k]
    assert one("12sha256_lanesE")["VGPRs"] <= 128
    assert one("17sha256_lanes_waitE")["VGPRs"] <= 128
    assert one("19sha256_b64dec_lanesE")["VGPRs"] <= 128
    assert one("16sha256_lanes_b64E")["VGPRs"] <= 168


def check_dpp_reads(ins):
    """Number of DPP instructions checked; raises on a DPP source written by a
    VALU instruction fewer than two wait states earlier."""
    checked = 0
    for i, (mn, ops) in enumerate(ins):
        if "_dpp" not in mn:
            continue
        # v_add_u32_dpp vdst, vsrc0 (permuted), vsrc1 <dpp controls>
        src0 = vregs(ops[1])
        assert src0, (mn, ops)
        waits, j = 0, i - 1
        while j >= 0 and waits < 2:
            pm, pops = ins[j]
            if pm.startswith("v_") and pops and vregs(pops[0]) & src0:
                raise AssertionError(f"{pm} {pops} writes the DPP source of {mn} {ops} {waits} wait states earlier")
            m = pm == "s_nop" and re.fullmatch(r"(\d+)", pops[0])
            waits += int(m.group(1)) + 1 if m else 1
            j -= 1
        checked += 1
    return checked


def test_pair_lane_kernel_keeps_the_dpp_read_hazard(device_asm):
    kernels = instructions(device_asm, "sha256_chain2")
    assert len(kernels) >= 2  # one and two wave pairs per workgroup
    # 3 DPP adds per round x 64 rounds (+ the block's first) per instantiation
    assert sum(check_dpp_reads(ins) for ins in kernels) >= 2 * 193


GOOD = """
k_test:
	v_add3_u32 v5, v5, v6, v4
	v_add_u32_dpp v3, v3, v5 row_shl:4 row_mask:0xf bank_mask:0x5
	v_add_u32_dpp v4, v2, v12 quad_perm:[0,1,2,3] row_mask:0xf bank_mask:0x5
	v_add_u32_dpp v3, v5, v5 row_shr:4 row_mask:0xf bank_mask:0xa
	s_endpgm
"""


def test_the_checker_sees_a_violation():
    (ins,) = instructions(GOOD, "k_test")
    assert check_dpp_reads(ins) == 3
    # one wait state only between the add3 and the DPP read of its result
    (bad,) = instructions(GOOD.replace("\tv_add_u32_dpp v4, v2, v12 quad_perm:[0,1,2,3] row_mask:0xf bank_mask:0x5\n", ""),
                          "k_test")
    with pytest.raises(AssertionError):
        check_dpp_reads(bad)
    # ... and an s_nop 0 in its place repairs it, a written register range counts too
    (ok,) = instructions(GOOD.replace("v_add_u32_dpp v4, v2, v12 quad_perm:[0,1,2,3] row_mask:0xf bank_mask:0x5",
                                      "s_nop 0"), "k_test")
    assert check_dpp_reads(ok) == 2
    (rng,) = instructions(GOOD.replace("v_add3_u32 v5, v5, v6, v4", "v_lshlrev_b64 v[2:3], 1, v[8:9]"), "k_test")
    with pytest.raises(AssertionError):
        check_dpp_reads(rng)


def test_pair_lane_rounds_are_ten_instructions(device_asm):
    """The point of the kernel: 10 VALU instructions per round in the owner
    wave's block loop (3 rotates, 3 bit ops, one 3-operand add, 3 DPP adds),
    with no padding between them."""
    for ins in instructions(device_asm, "sha256_chain2"):
        first = next(i for i, (mn, _) in enumerate(ins) if "_dpp" in mn)
        last = max(i for i, (mn, _) in enumerate(ins) if "_dpp" in mn)
        body = ins[first:last + 1]
        n_dpp = sum("_dpp" in mn for mn, _ in body)
        assert n_dpp == 193
        valu = sum(mn.startswith("v_") for mn, _ in body)
        nops = sum(mn == "s_nop" for mn, _ in body)
        assert valu <= 64 * 10 + 16, valu   # the rounds, plus a few copies the register allocator adds
        assert nops <= 2, nops


@pytest.mark.parametrize("name", ["base64.hip", "gather.hip"])
def test_stream_kernels_do_not_spill(tmp_path, name):
    """The HBM-bound kernels: no scratch, no spills; the Base64 encode kernel
    stays within the 64 VGPRs that let two of its workgroups per CU sit beside
    three SHA waves per SIMD (3 x 128 + 2 x 64 <= 512)."""
    if not os.path.exists(HIPCC):
        pytest.skip("no hipcc")
    _, remarks = compile_device(os.path.join(os.path.dirname(SRC), name), tmp_path / (name + ".s"))
    res = resources(remarks)
    assert res, remarks[-500:]
    for k, v in res.items():
        assert v["ScratchSize"] == 0 and v["VGPRs Spill"] == 0, (k, v)
    if name == "base64.hip":
        (enc,) = [v for k, v in res.items() if "b64_encode_kernel" in k]
        assert enc["VGPRs"] <= 64, enc
