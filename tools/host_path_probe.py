"""Per-call time of pcppx_parse_batch_host under the record options the facade's reader pages have used (GPU box, repo
root): round 4's pages (FIXED 16 rows + the 32-B summary, checksums on) against round 5's (the brief + DENSE chains,
checksums as the caller asked: off for Packet(&raw, TCP)), and the two mixed forms, on the reference's example.pcap
(frozen in tests/golden/capture_example.npz), BASELINE config 1's 10k packets and a 1M-packet config-3 page. Outputs are
page-locked (as the facade's PinnedPool records: the D2H lands in them directly); each call's median over `reps` calls,
the forms interleaved call by call.

  python tools/host_path_probe.py [reps]
"""
from __future__ import annotations

import ctypes as C
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from pcapplusplus_amd import abi, synth  # noqa: E402
from pcapplusplus_amd.engine import Engine, PinnedBuffer  # noqa: E402

FORMS = {
    # name: (layout, brief instead of summary, checksums)
    "r04_fixed16_summary_csum": (abi.LAYOUT_FIXED, False, True),
    "r05_dense_brief": (abi.LAYOUT_DENSE, True, False),
    "fixed16_brief": (abi.LAYOUT_FIXED, True, False),
    "dense_summary_csum": (abi.LAYOUT_DENSE, False, True),
}


def main() -> None:
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    from conftest import GOLDEN, load_golden

    ex, _ = load_golden(GOLDEN / "capture_example.npz")
    batches = {"example.pcap": ex, "config1_10k": synth.config(1), "config3_1M": synth.config(3, 1_000_000)}
    out = {}
    with Engine(0) as eng:
        for bname, b in batches.items():
            n, ml = b.n, 16
            head = PinnedBuffer(n * 32)
            lay = PinnedBuffer(n * ml * 8)
            cb = b.c_batch()
            calls = {}
            for fname, (layout, brief, csum) in FORMS.items():
                o = abi.make_opts(0, 8, csum, ml, layout=layout)
                rec = abi.Records(None if brief else head.ptr, lay.ptr)
                if brief:
                    rec.brief = head.ptr
                calls[fname] = (o, rec)
            times = {f: [] for f in FORMS}
            for r in range(reps + 3):
                for fname, (o, rec) in calls.items():
                    t = time.perf_counter()
                    abi.check(eng.lib.pcppx_parse_batch_host(eng.ctx, C.byref(cb), C.byref(o), C.byref(rec)),
                              "pcppx_parse_batch_host")
                    dt = time.perf_counter() - t
                    if r >= 3:
                        times[fname].append(dt * 1e3)
            out[bname] = {"packets": n, **{f: {"median_ms": round(float(np.median(t)), 4),
                                               "min_ms": round(float(np.min(t)), 4)} for f, t in times.items()}}
            print(bname, json.dumps(out[bname]), flush=True)
            head.free()
            lay.free()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
