"""Extract the reference's golden simulation captures into a compact frame fixture.

Source: /root/reference/unit-test/exp/*.json — the recorded {"meta": "tx"|"rx",
"data": K12 hex} frames the reference's plugin simulation tests compare against
(src/emu/core/thread_ctx.go:309-324, veth.go:235-247).  This is data only: the frame bytes
and where they came from.  Run here (the reference is not on the GPU box):

    python tests/golden/make_corpus.py

Writes tests/golden/corpus_frames.npz with
    data  uint8[]   all frames concatenated
    off   uint32[]  frame start in data
    len   uint16[]  frame length
    meta  uint8[]   0 = tx, 1 = rx (frames the plugins answered: each reached a callback)
    src   uint16[]  index into `files`
    files str[]     source capture names
"""
import json
import sys
from pathlib import Path

import numpy as np

REF = Path("/root/reference/unit-test/exp")
OUT = Path(__file__).resolve().parent / "corpus_frames.npz"


def walk(x, out):
    if isinstance(x, dict):
        if x.get("meta") in ("tx", "rx") and isinstance(x.get("data"), str):
            out.append(x)
        for v in x.values():
            walk(v, out)
    elif isinstance(x, list):
        for v in x:
            walk(v, out)


def main():
    files = sorted(p for p in REF.glob("*.json"))
    data, off, ln, meta, fidx, names = bytearray(), [], [], [], [], []
    for fi, p in enumerate(files):
        names.append(p.name)
        try:
            doc = json.loads(p.read_text())
        except Exception as e:  # noqa: BLE001
            print("skip", p.name, e, file=sys.stderr)
            continue
        recs = []
        walk(doc, recs)
        for r in recs:
            b = bytes(int(h, 16) for h in r["data"].split("|") if h)
            if "len" in r:
                assert int(r["len"]) == len(b), (p.name, r["len"], len(b))
            off.append(len(data))
            ln.append(len(b))
            meta.append(1 if r["meta"] == "rx" else 0)
            fidx.append(fi)
            data += b
    np.savez_compressed(OUT, data=np.frombuffer(bytes(data), np.uint8), off=np.array(off, np.uint32),
                        len=np.array(ln, np.uint16), meta=np.array(meta, np.uint8),
                        src=np.array(fidx, np.uint16), files=np.array(names))
    m = np.array(meta)
    print(f"{len(off)} frames ({int(m.sum())} rx, {int((m == 0).sum())} tx), {len(data)} bytes "
          f"from {len(files)} captures -> {OUT}")


if __name__ == "__main__":
    main()
