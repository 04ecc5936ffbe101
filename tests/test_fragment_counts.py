"""Fragment counts away from the reference's N = 5 (and the bench's 8), in
batches big enough for the persistent SHA kernel and the decode-ahead
download: N = 1 (the whole file is its one fragment, a twin of its fileId
lane), N = 2, N = 48 (the most fragment groups one decode-ahead launch
tracks), N = 49 and 64 (beyond it: the download falls back to passes) and
N = 100 (more fragments than most files have bytes: SN:141-157 then yields
empty fragments).  Upload against the oracle (SN:127, 159, 636), download with
a wrong fragment digest, a wrong fileId and a missing fragment (SN:250-257,
443-446, 454-458)."""
import base64
import hashlib

import numpy as np
import pytest

import dfs_amd
import oracle as O
from test_twin_lanes import _check_upload, _files

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nfrag,nfiles", [(1, 34000), (2, 17000), (48, 700), (49, 700), (64, 520), (100, 340)])
def test_upload_and_download_with_n_fragments(engine, nfrag, nfiles):
    rng = np.random.default_rng(1000 + nfrag)
    sizes = rng.integers(0, 3000, nfiles)
    sizes[:6] = [0, 1, nfrag - 1, nfrag, nfrag + 1, 64 * nfrag]
    files = _files(sizes, nfrag)
    print(f"N = {nfrag}: {nfiles} files, {nfiles * (nfrag + 1)} SHA lanes", flush=True)
    ups = _check_upload(engine, files, nfrag)
    texts = [[g.b64 for g in u.fragments] for u in ups]
    frag_h = [[g.hash for g in u.fragments] for u in ups]
    file_h = [u.file_id for u in ups]
    for f in (0, 1, 2, 7, nfiles - 1):  # the upload's own output is what a download is given: spot-check it here
        parts = [files[f][o:o + n] for o, n in O.c_split(len(files[f]), nfrag)]
        assert texts[f] == [base64.b64encode(p) for p in parts] and file_h[f] == hashlib.sha256(files[f]).hexdigest()
    want = [0] * nfiles
    frag_h[10] = list(frag_h[10]); frag_h[10][nfrag - 1] = "0" * 64
    want[10] = dfs_amd.DFS_E_FRAG_MISMATCH
    file_h[20] = "f" * 64
    want[20] = dfs_amd.DFS_E_CORRUPT
    texts[30] = list(texts[30]); texts[30][nfrag // 2] = None
    want[30] = dfs_amd.DFS_E_MISSING
    res = engine.download(texts, [len(d) for d in files], frag_h, file_h)
    assert engine.stats()["ovl_redo"] == 0
    for f, (st, body) in enumerate(res):
        assert st == want[f], f
        if want[f] == 0:
            assert body == files[f], f
