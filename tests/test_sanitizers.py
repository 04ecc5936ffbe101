"""Host code under the sanitizers, on the CPU: the request batcher's thread
hand-off (csrc/batcher.cpp against host stand-ins for its HIP and compute
calls) and the fragment store's staging ring and I/O pool
(csrc/fragstore.cpp, same stand-ins) under ThreadSanitizer and under
AddressSanitizer + UBSan; the placement schedules, the simulated runner, the
replica layout and the host-staged communicator's mailboxes under
AddressSanitizer + UBSan.  Skipped where g++ has no sanitizer runtimes."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.timeout(900)


def _has_sanitizer(flag, tmp_path):
    src = tmp_path / "probe.cpp"
    src.write_text("int main() { return 0; }\n")
    p = subprocess.run(["g++", f"-fsanitize={flag}", str(src), "-o", str(tmp_path / "probe")], capture_output=True)
    return p.returncode == 0


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_batcher_handoff_under_tsan_and_asan(tmp_path):
    if not (_has_sanitizer("thread", tmp_path) and _has_sanitizer("address,undefined", tmp_path)):
        pytest.skip("g++ without sanitizer runtimes")
    env = dict(os.environ, OUT=str(tmp_path), THREADS="16", ITERS="10", DEPTH="2")
    p = subprocess.run(["bash", os.path.join(ROOT, "tools", "batcher_sanitize.sh")], capture_output=True, text=True,
                       env=env, timeout=800)
    out = p.stdout + p.stderr
    assert p.returncode == 0, out[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("batcher_sanitize_drv:")]
    assert len(lines) == 2 and all(ln.endswith(" 0 failed checks") for ln in lines), out[-3000:]
    assert "Sanitizer" not in out, out[-3000:]


@pytest.mark.skipif(shutil.which("g++") is None or not os.path.exists("/opt/rocm/lib/libamdhip64.so"),
                    reason="needs g++ and the HIP runtime library to link")
def test_placement_and_replica_layout_under_asan(tmp_path):
    if not _has_sanitizer("address,undefined", tmp_path):
        pytest.skip("g++ without sanitizer runtimes")
    env = dict(os.environ, TMPDIR=str(tmp_path))
    p = subprocess.run(["bash", os.path.join(ROOT, "tools", "place_sanitize.sh")], capture_output=True, text=True, env=env,
                       timeout=800)
    out = p.stdout + p.stderr
    assert p.returncode == 0, out[-3000:]
    assert "runtime error" not in out and "AddressSanitizer" not in out, out[-3000:]


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_fragment_store_under_tsan_and_asan(tmp_path):
    if not (_has_sanitizer("thread", tmp_path) and _has_sanitizer("address,undefined", tmp_path)):
        pytest.skip("g++ without sanitizer runtimes")
    p = subprocess.run(["bash", os.path.join(ROOT, "tools", "fragstore_sanitize.sh")], capture_output=True, text=True,
                       env=dict(os.environ, OUT=str(tmp_path)), timeout=800)
    out = p.stdout + p.stderr
    assert p.returncode == 0, out[-3000:]
    assert out.count("fragstore_sanitize_drv: 0 failed checks") == 2 and "Sanitizer" not in out, out[-3000:]


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_reply_parser_fuzz_under_asan(tmp_path):
    if not _has_sanitizer("address,undefined", tmp_path):
        pytest.skip("g++ without sanitizer runtimes")
    p = subprocess.run(["bash", os.path.join(ROOT, "tools", "wire_sanitize.sh")], capture_output=True, text=True,
                       env=dict(os.environ, OUT=str(tmp_path)), timeout=600)
    out = p.stdout + p.stderr
    assert p.returncode == 0 and "wire_sanitize_drv: 200000 replies" in out, out[-3000:]
    assert "runtime error" not in out and "AddressSanitizer" not in out, out[-3000:]
