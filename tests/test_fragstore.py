"""On-disk fragment store (dfs_store_write_fragments / dfs_store_read_fragments)
against the oracle's restatement of StorageNode's Files.write / readAllBytes
(SN:147-149, 163-166, 273-285, 463-469).

Host-buffer mode is pure file I/O (no device), so it runs here on the CPU;
device-buffer mode (HBM <-> pinned staging ring <-> disk) is `-m gpu`."""
import hashlib
import os

import numpy as np
import pytest

import oracle as O
from dfs_amd import _lib as L
from dfs_amd.fragstore import FragmentStore, make_refs


def _files(rng, sizes):
    return [rng.integers(0, 256, s, dtype=np.uint8).tobytes() for s in sizes]


def _node_refs(files, nfrag, node):
    """The fragments node `node` keeps of every file (SN:143-145: {node, node+1}),
    packed back to back in one buffer, in (file, fragment) order."""
    blobs, off, ln, fi, idx, pos = [], [], [], [], [], 0
    for f, data in enumerate(files):
        spans = O.py_split(len(data), nfrag)
        for i in O.py_node_fragments(node, nfrag):
            o, l = spans[i]
            blobs.append(data[o:o + l])
            off.append(pos), ln.append(l), fi.append(f), idx.append(i)
            pos += l
    buf = np.frombuffer(b"".join(blobs) or b"\0", dtype=np.uint8).copy()
    return buf, make_refs(off, ln, fi, idx), blobs


def _digests(files):
    return np.frombuffer(b"".join(hashlib.sha256(d).digest() for d in files), dtype=np.uint8).reshape(-1, 32)


def _oracle_tree(tmp_path, files, nfrag, node):
    root = str(tmp_path / "oracle" / f"node-{node}")
    for data in files:
        fid = O.py_sha256_hex(data)
        spans = O.py_split(len(data), nfrag)
        for i in O.py_node_fragments(node, nfrag):
            o, l = spans[i]
            O.py_store_write(root, fid, i, data[o:o + l])
    return O.py_tree(root)


@pytest.mark.parametrize("slot_mb", ["64", "1"])
def test_host_write_matches_oracle_tree(tmp_path, monkeypatch, slot_mb):
    monkeypatch.setenv("DFS_STORE_SLOT_MB", slot_mb)  # 1 MiB: multi-chunk fragments
    rng = np.random.default_rng(7)
    sizes = [0, 1, 4, 5, 28, 467, 2154, 9506, 3 << 20, (5 << 20) + 3]
    files = _files(rng, sizes)
    for node in range(5):
        buf, refs, _ = _node_refs(files, 5, node)
        store = FragmentStore(node + 1, str(tmp_path / "ours"))
        st = store.write(_digests(files), buf, refs)
        assert (st == 0).all()
        assert O.py_tree(store.root) == _oracle_tree(tmp_path, files, 5, node)


def test_host_read_round_trip_and_missing(tmp_path, monkeypatch):
    monkeypatch.setenv("DFS_STORE_SLOT_MB", "1")
    rng = np.random.default_rng(11)
    files = _files(rng, [0, 100, 3 << 20, 777])
    buf, refs, blobs = _node_refs(files, 5, 2)
    store = FragmentStore(3, str(tmp_path))
    assert (store.write(_digests(files), buf, refs) == 0).all()
    back = np.zeros_like(buf)
    st, ln = store.read(_digests(files), back, refs)
    assert (st == 0).all() and list(ln) == [len(b) for b in blobs]
    assert back.tobytes() == buf.tobytes()
    # a fragment this node does not hold -> DFS_E_MISSING (tryLoadFragmentLocal null)
    miss = make_refs([0], [10], [1], [4])
    st, _ = store.read(_digests(files), back, miss)
    assert st[0] == L.DFS_E_MISSING
    fid = O.py_sha256_hex(files[1])
    assert store.try_load_fragment_local(fid, 4) is None
    assert store.try_load_fragment_local(fid, 2) == O.py_try_load_fragment_local(store.root, fid, 2)
    # capacity smaller than the file -> DFS_E_ARG, nothing else disturbed
    small = refs.copy()
    small["len"][3] = max(0, int(small["len"][3]) - 1)
    st, _ = store.read(_digests(files), back, small)
    assert st[3] == L.DFS_E_ARG and (np.delete(st, 3) == 0).all()


def test_overwrite_truncates(tmp_path):
    """Files.write(path, bytes) truncates an existing file (SN:166, 285)."""
    dig = _digests([b"x"])
    store = FragmentStore(1, str(tmp_path))
    long = np.arange(1000, dtype=np.uint8)
    store.write(dig, long, make_refs([0], [1000], [0], [0]))
    store.write(dig, long, make_refs([0], [10], [0], [0]))
    fid = dig[0].tobytes().hex()
    assert O.py_try_load_fragment_local(store.root, fid, 0) == long[:10].tobytes()


def test_reference_examples_layout(tmp_path, example_bytes):
    """Node 1 uploads examples/* with N=5 and keeps fragments {0, 1}
    (SN:143-145); the paths and bytes are the reference's."""
    names = sorted(example_bytes)
    files = [example_bytes[n] for n in names]
    buf, refs, blobs = _node_refs(files, 5, 0)
    store = FragmentStore(1, str(tmp_path / "data"))
    assert (store.write(_digests(files), buf, refs) == 0).all()
    for f, data in enumerate(files):
        fid = hashlib.sha256(data).hexdigest()
        spans = O.py_split(len(data), 5)
        for i in (0, 1):
            p = os.path.join(str(tmp_path), "data", "node-1", fid, "fragments", f"{i}.frag")
            o, l = spans[i]
            assert open(p, "rb").read() == data[o:o + l]


def test_bad_arguments(tmp_path):
    lib = L.lib()
    dig = np.zeros(32, dtype=np.uint8)
    refs = make_refs([0], [4], [0], [0])
    st = np.zeros(1, dtype=np.int32)
    # device pointers without a ctx, NULL root, NULL data with a non-empty ref
    assert lib.dfs_store_write_fragments(None, str(tmp_path).encode(), dig.ctypes.data, 1, None, refs.ctypes.data, 1,
                                         st.ctypes.data, L.DFS_DEVICE_PTRS) == L.DFS_E_ARG
    assert lib.dfs_store_write_fragments(None, None, dig.ctypes.data, 1, None, refs.ctypes.data, 1, st.ctypes.data,
                                         0) == L.DFS_E_ARG
    assert lib.dfs_store_read_fragments(None, str(tmp_path).encode(), dig.ctypes.data, 1, None, refs.ctypes.data, 1,
                                        None, st.ctypes.data, 0) == L.DFS_E_ARG
    # a ref naming a file past the digest table: rejected before any I/O
    data4 = np.zeros(4, dtype=np.uint8)
    bad = make_refs([0], [4], [1], [0])
    assert lib.dfs_store_write_fragments(None, str(tmp_path).encode(), dig.ctypes.data, 1, data4.ctypes.data,
                                         bad.ctypes.data, 1, st.ctypes.data, 0) == L.DFS_E_ARG
    assert lib.dfs_store_read_fragments(None, str(tmp_path).encode(), dig.ctypes.data, 1, data4.ctypes.data,
                                        bad.ctypes.data, 1, None, st.ctypes.data, 0) == L.DFS_E_ARG
    assert not any(tmp_path.iterdir())
    # a path component that is a file -> DFS_E_IO (createDirectories throws)
    blocker = tmp_path / "blk"
    blocker.write_bytes(b"")
    data = np.zeros(4, dtype=np.uint8)
    assert lib.dfs_store_write_fragments(None, str(blocker).encode(), dig.ctypes.data, 1, data.ctypes.data,
                                         refs.ctypes.data, 1, st.ctypes.data, 0) == L.DFS_E_IO
    assert st[0] == L.DFS_E_IO


@pytest.mark.gpu
@pytest.mark.parametrize("slot_mb", ["64", "1"])
def test_device_store_round_trip(tmp_path, monkeypatch, engine, slot_mb):
    """HBM -> pinned ring -> disk and back, bit-exact vs the oracle's tree;
    1 MiB slots exercise multi-chunk fragments and ring reuse."""
    import torch
    monkeypatch.setenv("DFS_STORE_SLOT_MB", slot_mb)
    rng = np.random.default_rng(5)
    files = _files(rng, [0, 3, 28, 9506, 2154, 467, (3 << 20) + 1] + [200_000] * 40)
    dig = _digests(files)
    buf, refs, blobs = _node_refs(files, 5, 4)
    d_buf = torch.from_numpy(buf).to("cuda:0")
    store = FragmentStore(5, str(tmp_path / "ours"), engine=engine)
    st = store.write(dig, d_buf.data_ptr(), refs, device=True)
    assert (st == 0).all()
    assert O.py_tree(store.root) == _oracle_tree(tmp_path, files, 5, 4)
    d_back = torch.zeros_like(d_buf)
    torch.cuda.synchronize()  # torch filled these on its stream; the library runs on the engine's
    st, ln = store.read(dig, d_back.data_ptr(), refs, device=True)
    assert (st == 0).all() and list(ln) == [len(b) for b in blobs]
    assert d_back.cpu().numpy().tobytes() == buf.tobytes()


@pytest.mark.gpu
def test_device_config1_download_from_disk(tmp_path, engine, example_bytes):
    """BASELINE config 1 with the disk in the loop: node 1 uploads examples/*
    (+ a 1 MiB file), every node stores its pair from HBM (SN:163-166,
    284-285), node 3 goes down, node 1 downloads: local fragments from its
    own store, the rest from the first live holder's store (SN:421-451),
    read straight into HBM, then gather + fileId verify on the device
    (SN:454-458)."""
    import torch
    from dfs_amd.engine import reassemble_device
    N, down, me = 5, 2, 0
    files = [example_bytes[n] for n in sorted(example_bytes)] + [O.c_synth(3, 0, 1 << 20)]
    ups = engine.upload(files, N)
    dig = np.frombuffer(b"".join(bytes.fromhex(u.file_id) for u in ups), dtype=np.uint8).reshape(-1, 32)
    S = [len(x) for x in files]
    base = np.concatenate([[0], np.cumsum(S)[:-1]]).astype(np.uint64)
    d_files = torch.from_numpy(np.frombuffer(b"".join(files), dtype=np.uint8).copy()).to("cuda:0")
    spans = [O.py_split(s, N) for s in S]
    stores = [FragmentStore(k + 1, str(tmp_path / "data"), engine=engine) for k in range(N)]
    for k in range(N):
        off, ln, fi, ix = [], [], [], []
        for f in range(len(files)):
            for i in O.py_node_fragments(k, N):
                o, l = spans[f][i]
                off.append(int(base[f]) + o), ln.append(l), fi.append(f), ix.append(i)
        assert (stores[k].write(dig, d_files.data_ptr(), make_refs(off, ln, fi, ix), device=True) == 0).all()
    # download plan (SN:421-451): local first, then holders in order, node `down` offline
    d_frag = torch.zeros(sum(S) + 64, dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()  # torch filled these on its stream; the library runs on the engine's
    addr = np.zeros(len(files) * N, dtype=np.uint64)
    flen = np.zeros(len(files) * N, dtype=np.uint64)
    per_node = {}
    for f in range(len(files)):
        for i in range(N):
            src = me if i in O.py_node_fragments(me, N) else next(h for h in O.py_fragment_holders(i, N) if h != down)
            o, l = spans[f][i]
            per_node.setdefault(src, []).append((int(base[f]) + o, l, f, i))
            addr[f * N + i] = d_frag.data_ptr() + int(base[f]) + o
            flen[f * N + i] = l
    for src, items in per_node.items():
        off, ln, fi, ix = zip(*items)
        st, got = stores[src].read(dig, d_frag.data_ptr(), make_refs(off, ln, fi, ix), device=True)
        assert (st == 0).all() and list(got) == list(ln)
    d_out = torch.zeros(sum(S) + 64, dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()  # torch filled these on its stream; the library runs on the engine's
    st, fdig = reassemble_device(engine, addr, flen, len(files), N, d_out.data_ptr(), base, expected=dig)
    assert (st == 0).all() and (fdig == dig).all()
    assert d_out[:sum(S)].cpu().numpy().tobytes() == b"".join(files)
