"""Single-request latency of the fragment pipeline (one 1 MiB upload and one
download through the C ABI, host buffers) and the SHA kernel time of that
launch (HIP events).  Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-file-storage_amd"))
import dfs_amd  # noqa: E402


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    eng = dfs_amd.FragmentEngine(0)
    data = np.random.default_rng(1).integers(0, 256, S, dtype=np.uint8).tobytes()
    up = eng.upload([data], 5)
    eng.set_profiling(True)
    wall, sha = [], []
    for _ in range(20):
        t0 = time.perf_counter()
        up = eng.upload([data], 5)
        wall.append(time.perf_counter() - t0)
        sha.append(eng.timings()["sha"])
    dwall = []
    texts = [[g.b64 for g in up[0].fragments]]
    for _ in range(20):
        t0 = time.perf_counter()
        res = eng.download(texts, [S], [[g.hash for g in up[0].fragments]], [up[0].file_id])
        dwall.append(time.perf_counter() - t0)
        assert res[0][0] == 0 and res[0][1] == data
    print(json.dumps({"file_bytes": S, "upload_wall_ms_p50": round(float(np.median(wall)) * 1e3, 3),
                      "upload_sha_kernel_ms_p50": round(float(np.median(sha)), 3),
                      "download_wall_ms_p50": round(float(np.median(dwall)) * 1e3, 3)}))
    eng.close()


if __name__ == "__main__":
    main()
