"""Twin lanes (kShaTwin, sha256.hip / dfs_gpu.cpp add_lane_with_twins): a
fragment that starts on the 64-byte block grid of its file's fileId lane rides
in that lane — one load and one message schedule per block for both digests.
That is fragment 0 of every file (SN:153, offset 0) and every fragment when the
fragment size is a multiple of 64 (BASELINE configs[2]: 256 KiB, N = 8).
Twins are built only for launches that keep at least dfs::kTwinMinLanes
(65,536) lanes, one wave per SIMD, so every batch here has that many.  Bit-exact against the oracle
(fileId SN:127, fragment digests SN:159, Base64 SN:636) and, on download,
decode + fragment verify + fileId verify (SN:281-282, 448-458).
"""
import base64
import hashlib

import numpy as np
import pytest

import dfs_amd
import oracle as O

pytestmark = pytest.mark.gpu


def _files(sizes, seed):
    rng = np.random.default_rng(seed)
    blob = rng.integers(0, 256, int(sum(sizes)), dtype=np.uint8).tobytes()
    out, o = [], 0
    for n in sizes:
        out.append(blob[o:o + int(n)])
        o += int(n)
    return out


def _check_upload(engine, files, nfrag):
    ups = engine.upload(files, nfrag)
    fd, frd, b64, off = O.c_upload_batch(files, nfrag)
    for f, u in enumerate(ups):
        assert u.file_id == fd[f].tobytes().hex(), f
        for i, g in enumerate(u.fragments):
            assert g.hash == frd[f, i].tobytes().hex(), (f, i)
            k = f * nfrag + i
            assert g.b64 == b64[int(off[k]):int(off[k + 1])], (f, i)
    return ups


# (files, file size, N): every fragment a twin (256 B fragments, 8 per file);
# fragment 0 only (N = 5, 200-byte fragments start at 200, 400, ...: off the
# grid); every fragment exactly one block; fragment 0 one block + 1 byte (the
# others start off the grid).
SHAPES = [(66000, 2048, 8), (40000, 1000, 5), (66000, 320, 5), (34000, 324, 5)]


@pytest.mark.parametrize("nfiles,size,nfrag", SHAPES)
def test_twin_upload_uniform(engine, nfiles, size, nfrag):
    _check_upload(engine, _files([size] * nfiles, nfiles + size), nfrag)


def test_twin_upload_ragged(engine):
    """Waves whose lanes have different twin lists (count, first block, tail
    bytes) and lanes without twins, sorted together: sizes 256*k (all four
    fragments twins), 256*k + 1..3 (fragment 0 only, with a 1-byte or longer
    tail), random sizes, < 64-byte fragments (no twin) and empty files."""
    rng = np.random.default_rng(5)
    n = 36000
    sizes = rng.integers(0, 6000, n)  # 36,000 fileId lanes + the fragments that are not twins
    sizes[0::5] = 256 * rng.integers(1, 24, len(sizes[0::5]))
    sizes[1::5] = 256 * rng.integers(1, 24, len(sizes[1::5])) + rng.integers(1, 4, len(sizes[1::5]))
    sizes[2::97] = rng.integers(0, 256, len(sizes[2::97]))
    sizes[3::1001] = 0
    _check_upload(engine, _files(sizes, 6), 4)


@pytest.mark.parametrize("mode", ["overlap", "pipelined", "serial"])
@pytest.mark.parametrize("nfiles,size,nfrag", [(66000, 2048, 8), (40000, 1000, 5)])
def test_twin_download(engine, mode, nfiles, size, nfrag, monkeypatch):
    """Download of twin-shaped batches: overlap (one SHA launch beside the
    fragment-ordered decode; twins inside the fileId lane's wait segments),
    pipelined (pass p's fileId part carries the group's on-grid fragments as
    twins) and serial (one launch), every file rebuilt and verified, plus a
    wrong fragment digest on a twin (fragment 0) and on a non-twin, and a
    wrong fileId."""
    if mode != "overlap":
        monkeypatch.setenv("DFS_DOWNLOAD_MODE", mode)
        engine = dfs_amd.FragmentEngine(0)
    try:
        files = _files([size] * nfiles, 3 * nfiles + size)
        texts, frag_h, file_h = [], [], []
        for d in files:
            parts = [d[o:o + n] for o, n in O.c_split(len(d), nfrag)]
            texts.append([base64.b64encode(p) for p in parts])
            frag_h.append([hashlib.sha256(p).hexdigest() for p in parts])
            file_h.append(hashlib.sha256(d).hexdigest())
        want = [0] * nfiles
        frag_h[10] = list(frag_h[10]); frag_h[10][0] = "0" * 64
        want[10] = dfs_amd.DFS_E_FRAG_MISMATCH
        frag_h[20] = list(frag_h[20]); frag_h[20][nfrag - 1] = "1" * 64
        want[20] = dfs_amd.DFS_E_FRAG_MISMATCH
        file_h[nfiles - 1] = "f" * 64
        want[nfiles - 1] = dfs_amd.DFS_E_CORRUPT
        res = engine.download(texts, [len(d) for d in files], frag_h, file_h)
        assert engine.stats()["ovl_redo"] == 0  # no decode-ahead wait timed out
    finally:
        if mode != "overlap":
            engine.close()
    for f, (st, body) in enumerate(res):
        assert st == want[f], f
        if want[f] == 0:
            assert body == files[f], f


@pytest.fixture(scope="module")
def hybrid_engine():
    """DFS_UPLOAD_MODE=hybrid: the fragment lanes write their own Base64 in the
    SHA pass and the encode kernel covers only the twins."""
    import os
    old = os.environ.get("DFS_UPLOAD_MODE")
    os.environ["DFS_UPLOAD_MODE"] = "hybrid"
    try:
        eng = dfs_amd.FragmentEngine(0)
    finally:
        if old is None:
            del os.environ["DFS_UPLOAD_MODE"]
        else:
            os.environ["DFS_UPLOAD_MODE"] = old
    yield eng
    eng.close()


@pytest.mark.parametrize("nfiles,size,nfrag", SHAPES + [(33000, 4099, 5), (300, 70001, 3)])
def test_hybrid_upload_uniform(hybrid_engine, nfiles, size, nfrag):
    """Digests and Base64 of the hybrid upload against the oracle: launches with
    twins (fragment 0, or every fragment) beside encoding fragment lanes, and
    a small launch without twins (every fragment encoded by its own lane)."""
    _check_upload(hybrid_engine, _files([size] * nfiles, nfiles + size + 1), nfrag)


def test_hybrid_upload_ragged(hybrid_engine):
    rng = np.random.default_rng(15)
    n = 36000
    sizes = rng.integers(0, 6000, n)
    sizes[0::5] = 256 * rng.integers(1, 24, len(sizes[0::5]))
    sizes[1::5] = 256 * rng.integers(1, 24, len(sizes[1::5])) + rng.integers(1, 4, len(sizes[1::5]))
    sizes[2::97] = rng.integers(0, 256, len(sizes[2::97]))
    sizes[3::1001] = 0
    _check_upload(hybrid_engine, _files(sizes, 16), 4)


@pytest.mark.parametrize("align128,frag_major", [(True, False), (False, True), (True, True)])
def test_hybrid_upload_plan_device(hybrid_engine, align128, frag_major):
    """The prepared plan on device buffers (the bench's path) in hybrid mode,
    1 MiB-like geometry scaled down (fragments 1.. off the block grid): every
    fileId, fragment digest and fragment Base64 (through its SHA-256) against
    the oracle's C path over the same synthetic files; also without fileIds
    (every fragment lane encodes, no encode kernel)."""
    import torch
    from dfs_amd.engine import sha256_device
    nfiles, S, nfrag = 70000, 5 * 211 + 1, 5
    spans = np.array([(f * S, S) for f in range(nfiles)], dtype=np.uint64)
    files = torch.empty(nfiles * S + 64, dtype=torch.uint8, device="cuda")
    dfs_amd.synth_fill(hybrid_engine, files.data_ptr(), spans, 31000, O.SYNTH_SEED)
    plan = dfs_amd.UploadPlan(hybrid_engine, spans, nfrag, frag_major=frag_major, align128=align128)
    efd, efrd, eb64 = O.synth_digests(31000, nfiles, S, nfrag, 8)
    try:
        for flags in (0, dfs_amd.DFS_NO_FILEID):
            fd = torch.zeros(nfiles * 32, dtype=torch.uint8, device="cuda")
            frd = torch.zeros(nfiles * nfrag * 32, dtype=torch.uint8, device="cuda")
            b64 = torch.zeros(plan.b64_total + 64, dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()  # torch filled these on its stream; the library runs on the engine's
            plan.run(files.data_ptr(), fd.data_ptr(), frd.data_ptr(), b64.data_ptr(), flags)
            torch.cuda.synchronize()
            if not flags:
                assert (fd.view(nfiles, 32).cpu().numpy() == efd).all()
            assert (frd.view(nfiles, nfrag, 32).cpu().numpy() == efrd).all()
            got = sha256_device(hybrid_engine, b64.data_ptr(), plan.b64_spans([S] * nfiles)).reshape(nfiles, nfrag, 32)
            bad = np.argwhere((got != eb64).any(axis=2))
            assert bad.size == 0, (flags, bad[:5].tolist())
    finally:
        plan.close()
