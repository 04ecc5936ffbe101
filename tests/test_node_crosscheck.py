"""A third implementation beside the oracle's two: Node.js (its own Base64
codec, `crypto` SHA-256) computes the upload half of the example files and of
seeded synthetic files — fileId, fragment digests and fragment Base64 after
the reference's split (StorageNode.java:138-171, 159, 636) — and the oracle's
C path must agree byte for byte.  Not the JDK (none exists here), so parity
with the reference stays unpinned; this only shows that the restatement
agrees with every independent codec at hand.  Skipped without `node`."""
import json
import os
import shutil
import subprocess

import pytest

import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))

NODE_SCRIPT = r"""
const crypto = require('crypto');
const fs = require('fs');
const req = JSON.parse(fs.readFileSync(0, 'utf8'));
const out = [];
for (const item of req.items) {
  const buf = item.path ? fs.readFileSync(item.path) : Buffer.from(item.hex, 'hex');
  const n = req.nfrag, total = buf.length;
  const base = Math.floor(total / n), rem = total % n;       // the split of handleUpload
  const frags = [];
  let off = 0;
  for (let i = 0; i < n; i++) {
    const len = base + (i < rem ? 1 : 0);
    const part = buf.slice(off, off + len);
    frags.push({sha: crypto.createHash('sha256').update(part).digest('hex'), b64: part.toString('base64')});
    off += len;
  }
  out.push({file: crypto.createHash('sha256').update(buf).digest('hex'), frags});
}
process.stdout.write(JSON.stringify(out));
"""


@pytest.mark.skipif(shutil.which("node") is None, reason="no node")
@pytest.mark.parametrize("nfrag", [5, 8])
def test_oracle_agrees_with_node(nfrag, tmp_path):
    ex = os.path.join(HERE, "golden", "examples")
    items, datas = [], []
    for name in sorted(os.listdir(ex)):
        p = os.path.join(ex, name)
        items.append({"path": p})
        datas.append(open(p, "rb").read())
    for i, n in enumerate([0, 1, 2, 3, 4, 5, 7, 55, 56, 64, 119, 120, 1000, 4099, 65537]):
        d = O.c_synth(31337 + i, 0, n)
        items.append({"hex": d.hex()})
        datas.append(d)
    script = tmp_path / "upload.js"
    script.write_text(NODE_SCRIPT)
    p = subprocess.run(["node", str(script)], input=json.dumps({"nfrag": nfrag, "items": items}), capture_output=True,
                       text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    got = json.loads(p.stdout)
    fd, frd, b64, off = O.c_upload_batch(datas, nfrag)
    for f, g in enumerate(got):
        assert fd[f].tobytes().hex() == g["file"], f
        assert O.py_sha256_hex(datas[f]) == g["file"], f
        for k in range(nfrag):
            assert frd[f, k].tobytes().hex() == g["frags"][k]["sha"], (f, k)
            lo, hi = int(off[f * nfrag + k]), int(off[f * nfrag + k + 1])
            assert b64[lo:hi].decode() == g["frags"][k]["b64"], (f, k)
