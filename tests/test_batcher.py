"""Request batcher (dfs_batcher / dfs_submit_*): many handler threads, one file
each (StorageNode's thread-per-connection model, SN:28-31), coalesced into
batched launches.  Every result is checked bit-exact against the CPU oracle:
uploads (fileId, fragment digests, fragment Base64) and downloads (bytes,
and the reference's failure statuses)."""
import threading

import numpy as np
import pytest

import dfs_amd
import oracle as O
from dfs_amd.batcher import Batcher

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(120)]

SIZES = [0, 1, 2, 4, 5, 7, 28, 55, 56, 64, 119, 467, 2154, 9506, 65535, 1 << 20, (1 << 20) + 3, 3 << 20]


def _file(i):
    return O.c_synth(7000 + i, 0, SIZES[i % len(SIZES)] if i < 2 * len(SIZES) else 1000 + 37 * i)


def _run_threads(n, fn):
    errs = []
    start = threading.Barrier(n)

    def body(t):
        try:
            start.wait()
            fn(t)
        except Exception as e:  # collected, reported by the main thread
            import traceback
            errs.append(traceback.format_exc())
    ths = [threading.Thread(target=body, args=(t,)) for t in range(n)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(timeout=300)
    assert not errs, errs[0]


@pytest.mark.parametrize("nfrag", [5, 8])
def test_concurrent_uploads_and_downloads_vs_oracle(nfrag):
    threads, per = 64, 3
    with Batcher(0, nfrag, max_wait_us=2000) as b:
        results = {}

        def work(t):
            for k in range(per):
                i = t * per + k
                data = _file(i)
                fd, frd, texts = b.upload(data)
                efd, efrd, eb64, eoff = O.c_upload_batch([data], nfrag)
                assert fd == efd[0].tobytes(), i
                assert frd == [efrd[0, j].tobytes() for j in range(nfrag)], i
                assert b"".join(texts) == eb64, i
                st, back = b.download(texts, len(data), frd, fd)
                assert st == 0 and back == data, (i, st)
                results[i] = True
        _run_threads(threads, work)
        assert len(results) == threads * per
        s = b.stats()
        assert s["requests"] == 2 * threads * per
        assert s["batches"] < s["requests"]  # concurrent calls were coalesced
        assert s["max_batch"] > 1


def test_download_failure_statuses_and_mixed_expectations():
    nfrag = 5
    with Batcher(0, nfrag, max_wait_us=2000) as b:
        data = O.c_synth(42, 0, 100003)
        fd, frd, texts = b.upload(data)
        cases = []
        cases.append(("ok", texts, frd, fd, 0))
        cases.append(("no expectations", texts, None, None, 0))
        cases.append(("file digest only", texts, None, fd, 0))
        miss = list(texts)
        miss[2] = None
        cases.append(("missing", miss, frd, fd, dfs_amd.DFS_E_MISSING))       # SN:443-446
        bad = list(texts)
        bad[1] = bad[1][:10] + b"*" + bad[1][11:]
        cases.append(("bad char", bad, frd, fd, dfs_amd.DFS_E_DECODE))        # SN:281 IAE
        wrong = list(frd)
        wrong[3] = bytes(32)
        cases.append(("frag digest", texts, wrong, fd, dfs_amd.DFS_E_FRAG_MISMATCH))  # SN:250-257
        cases.append(("file digest", texts, frd, bytes(32), dfs_amd.DFS_E_CORRUPT))  # SN:455-458
        out = {}

        def work(t):
            name, tx, ef, ei, want = cases[t % len(cases)]
            st, back = b.download(tx, len(data), ef, ei)
            out[t] = (name, st, want, back == data if st == 0 else back is None)
        _run_threads(4 * len(cases), work)
        for t, (name, st, want, good) in out.items():
            assert st == want and good, (name, st, want)


def test_single_request_latency_path():
    """One handler alone: the batch of one still runs (window expires)."""
    with Batcher(0, 5, max_wait_us=100) as b:
        data = O.c_synth(3, 0, 1 << 20)
        fd, frd, texts = b.upload(data)
        efd, efrd, eb64, _ = O.c_upload_batch([data], 5)
        assert fd == efd[0].tobytes() and b"".join(texts) == eb64
        assert b.stats()["batches"] == 1


def test_direct_pinned_requests_mixed_with_staged():
    """Handlers whose buffers come from dfs_host_alloc (direct: the worker's
    DMA reads / writes them) share batches with handlers on pageable memory
    (staged); every result bit-exact vs the oracle, a failed download leaves
    the caller's output untouched in both modes."""
    from dfs_amd import _lib as L
    from dfs_amd.batcher import PinnedBuffer
    nfrag, threads, per = 5, 48, 3
    with Batcher(0, nfrag, max_wait_us=3000) as b:
        def work(t):
            direct = t % 2 == 0
            for k in range(per):
                i = t * per + k
                data = _file(i)
                n = len(data)
                efd, efrd, eb64, eoff = O.c_upload_batch([data], nfrag)
                cap = len(eb64) + 16
                if direct:
                    fin, bout = PinnedBuffer(max(n, 1)), PinnedBuffer(cap)
                    src, b64 = fin.array[:n], bout.array
                else:
                    src, b64 = np.frombuffer(data, np.uint8).copy(), np.zeros(cap, np.uint8)
                if direct:
                    src[:] = np.frombuffer(data, np.uint8)
                fd, frd, off = np.zeros(32, np.uint8), np.zeros((nfrag, 32), np.uint8), np.zeros(nfrag + 1, np.uint64)
                assert b.upload_into(src, fd, frd, b64, off) == 0, i
                assert fd.tobytes() == efd[0].tobytes() and frd.tobytes() == efrd[0].tobytes(), i
                assert b64[:int(off[nfrag])].tobytes() == eb64, i
                # download from the same (pinned or pageable) Base64, into a
                # (pinned or pageable) output; every third one corrupt
                spans = (L.dfs_span * nfrag)()
                for j in range(nfrag):
                    spans[j].off, spans[j].len = int(off[j]), int(off[j + 1] - off[j])
                bad = k == 2 and n > 0
                ei = np.frombuffer(bytes(32) if bad else fd.tobytes(), np.uint8)
                dout = PinnedBuffer(max(n, 1)) if direct else None
                out = dout.array if direct else np.zeros(max(n, 1), np.uint8)
                out[:] = 0xA5
                st = b.download_into(b64, spans, n, frd.reshape(-1), ei, out)
                if bad:
                    assert st == dfs_amd.DFS_E_CORRUPT and (out == 0xA5).all(), (i, st)
                else:
                    assert st == 0 and out[:n].tobytes() == data, (i, st)
                for pb in ([fin, bout, dout] if direct else []):
                    pb.free()
        _run_threads(threads, work)
        s = b.stats()
        assert s["requests"] == 2 * threads * per
        assert s["direct"] == threads * per  # half the handlers, uploads and downloads
        assert s["batches"] < s["requests"]


def test_host_alloc_registry():
    from dfs_amd import _lib as L
    import ctypes
    p = ctypes.c_void_p()
    assert L.lib().dfs_host_alloc(4096, ctypes.byref(p)) == 0 and p.value
    assert L.lib().dfs_host_free(ctypes.c_void_p(p.value + 8)) == dfs_amd.DFS_E_ARG  # not an allocation start
    assert L.lib().dfs_host_free(p) == 0
    assert L.lib().dfs_host_free(p) == dfs_amd.DFS_E_ARG  # already freed


def test_concurrent_raw_fragment_downloads_vs_oracle():
    """dfs_submit_reassemble: handleDownload as the reference has it (SN:419-458,
    raw fragments) from 48 handler threads at once, mixed with uploads in the
    same batcher: the rebuilt bytes and digest against hashlib, a corrupted
    fragment ("File corrupted", SN:455-458: the caller's buffer untouched), a
    missing one ("Could not retrieve fragment", SN:443-446), empty files."""
    import hashlib
    nfrag = 5
    with Batcher(0, nfrag, max_wait_us=2000) as b:
        def work(t):
            for k in range(3):
                i = t * 3 + k
                data = _file(i)
                frags = [data[o:o + n] for o, n in O.c_split(len(data), nfrag)]
                want = hashlib.sha256(data).digest()
                st, back, dig = b.reassemble(frags, want)
                assert st == 0 and back == data and dig == want, (i, st)
                if t % 3 == 0:  # uploads interleave with the downloads in the queue
                    fd, _, _ = b.upload(data)
                    assert fd == want
                if len(data) >= nfrag:
                    bad = list(frags)
                    bad[2] = bytes([bad[2][0] ^ 0x40]) + bad[2][1:]
                    st, back, dig = b.reassemble(bad, want)
                    assert st == dfs_amd.DFS_E_CORRUPT and back is None
                    assert dig == hashlib.sha256(b"".join(bad)).digest()
                    gone = list(frags)
                    gone[4] = None
                    st, back, dig = b.reassemble(gone, want)
                    assert st == dfs_amd.DFS_E_MISSING and back is None
                st, back, dig = b.reassemble(frags, None)  # nothing to compare with
                assert st == 0 and back == data and dig == want
        _run_threads(48, work)
        s = b.stats()
        assert s["requests"] >= 48 * 3 * 2 and s["max_batch"] > 1


def test_view_outputs_mixed_with_copies():
    """dfs_submit_upload_view / dfs_submit_download_view: the answer stays in
    the batch's pinned result buffer and the handler gets a pointer.  Handlers
    asking for views (pinned or pageable inputs) share batches with handlers
    that take copies; every result bit-exact vs the oracle; a failed download
    hands out no view."""
    from dfs_amd import _lib as L
    from dfs_amd.batcher import PinnedBuffer
    nfrag, threads, per = 5, 48, 3
    with Batcher(0, nfrag, max_wait_us=3000) as b:
        def work(t):
            kind = t % 3  # 0: pinned input + views, 1: pageable input + views, 2: copies
            for k in range(per):
                i = t * per + k
                data = _file(i)
                n = len(data)
                efd, efrd, eb64, eoff = O.c_upload_batch([data], nfrag)
                if kind == 2:
                    fd, frd, texts = b.upload(data)
                else:
                    pb = PinnedBuffer(max(n, 1)) if kind == 0 else None
                    src = pb.array[:n] if pb else np.frombuffer(data, np.uint8).copy()
                    if pb:
                        src[:] = np.frombuffer(data, np.uint8)
                    fd, frd, texts = b.upload_view(src)
                    if pb:
                        pb.free()
                assert fd == efd[0].tobytes() and frd == [efrd[0, j].tobytes() for j in range(nfrag)], i
                assert b"".join(texts) == eb64, i
                if kind == 2:
                    st, back = b.download(texts, n, frd, fd)
                    assert st == 0 and back == data, (i, st)
                    continue
                total = len(eb64)
                tb = PinnedBuffer(max(total, 1)) if kind == 0 else None
                text = tb.array if tb else np.zeros(max(total, 1), np.uint8)
                text[:total] = np.frombuffer(eb64, np.uint8)
                spans = (L.dfs_span * nfrag)()
                for j in range(nfrag):
                    spans[j].off, spans[j].len = int(eoff[j]), int(eoff[j + 1] - eoff[j])
                bad = k == 2 and n > 0
                ei = np.frombuffer(bytes(32) if bad else fd, np.uint8)
                st, back = b.download_view(text, spans, n, np.frombuffer(b"".join(frd), np.uint8), ei)
                if bad:
                    assert st == dfs_amd.DFS_E_CORRUPT and back is None, (i, st)
                else:
                    assert st == 0 and back == data, (i, st)
                if tb:
                    tb.free()
        _run_threads(threads, work)
        s = b.stats()
        assert s["requests"] == 2 * threads * per
        assert s["views"] == 2 * (threads // 3) * per * 2
        assert s["batches"] < s["requests"]


def test_view_kept_across_later_batches():
    """A view stays readable and unchanged while later batches run: a worker
    takes a result buffer again only after every view of it was released, and
    adds a buffer rather than wait for a handler that keeps its view (one
    worker here: the third batch would need the first batch's buffer)."""
    from dfs_amd import _lib as L
    with Batcher(0, 5, max_wait_us=100, depth=1) as b:
        d1, d2, d3 = (O.c_synth(900 + j, 0, 300000 + j) for j in range(3))
        want1 = O.c_upload_batch([d1], 5)[2]
        fd1, frd1, off1 = np.zeros(32, np.uint8), np.zeros((5, 32), np.uint8), np.zeros(6, np.uint64)
        import ctypes
        ptr, view1 = ctypes.c_void_p(), ctypes.c_void_p()
        a1 = np.frombuffer(d1, np.uint8)
        assert L.lib().dfs_submit_upload_view(b._b, a1.ctypes.data, a1.size, fd1.ctypes.data, frd1.ctypes.data,
                                              ctypes.byref(ptr), off1.ctypes.data, ctypes.byref(view1)) == 0
        try:
            assert ctypes.string_at(ptr.value, int(off1[5])) == want1
            for d in (d2, d3, d2, d3):  # later batches, through the other buffer(s)
                _, _, texts = b.upload_view(np.frombuffer(d, np.uint8))
                assert b"".join(texts) == O.c_upload_batch([d], 5)[2]
            assert ctypes.string_at(ptr.value, int(off1[5])) == want1  # still there, untouched
        finally:
            Batcher.release_view(view1)
        assert L.lib().dfs_view_release(view1) == dfs_amd.DFS_E_ARG  # nothing left to release
