"""A/B of the decode attention's v staging image: padded rows (product, QZ_ATTN_VPAD=4) vs unpadded
(QZ_ATTN_VPAD=0), both full kernels (QZ_ATTN_ABL=0 builds from scripts/dev/build_attn_abl.sh), at the
bench's decode shape, interleaved three times."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from attn_ablation import run  # noqa: E402

for rep in range(3):
    for name in ("0_nopad", "0"):
        r = run(name)
        print(json.dumps({"build": name, "rep": rep, **{k: v for k, v in r.items() if k != "abl"}}), flush=True)
