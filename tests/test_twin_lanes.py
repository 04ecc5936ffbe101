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
