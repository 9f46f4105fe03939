"""Dev measurement: does streaming the NEXT layer's weights into the Infinity Cache from a side stream
(core.prefetch_l3) shorten the decode layer chain?  (1) the 4096^2 GEMV b2b over 64 rotating copies
(537 MB, from HBM) vs 8 copies (67 MB, Infinity-Cache resident): what a resident weight is worth to
one launch; (2) bench.chain_roofline (8B, 32 layers over 8 rotating sets) without and with the side
stream at several prefetch grid sizes / depths; (3) the same for 70B if asked (--70b)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

for c in (64, 8):
    mean, med, b2b, floor, empty = bench.gemv_roofline(copies=c)
    print(json.dumps({"gemv4096_copies": c, "b2b_us": round(b2b, 3), "read_floor_us": round(floor, 3),
                      "event_mean_us": round(mean, 3)}), flush=True)
variants = [None, (256, 8), (512, 8), (256, 16), (1024, 4)]
for pf in variants:
    r = bench.chain_roofline(prefetch=pf)
    print(json.dumps({"prefetch": pf, "us_per_layer": r["us_per_layer"], "min": r["us_per_layer_min"],
                      "max": r["us_per_layer_max"], "frac": r["frac"]}), flush=True)
if "--70b" in sys.argv:
    for pf in (None, (512, 8)):
        r = bench.chain_roofline(prefetch=pf, model_name="llama3-70b")
        print(json.dumps({"model": "70b", "prefetch": pf, "us_per_layer": r["us_per_layer"]}), flush=True)
