#!/bin/bash
# round 6 (closing): the Llama-3-70B single-GPU decode bench line (config #5 at N = 1)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 700 python3 -u bench.py --model llama3-70b > gpurun_out/r6_bench70.json 2> gpurun_out/r6_bench70.err || { tail -5 gpurun_out/r6_bench70.err; exit 1; }
python3 -c "
import json; l=json.loads(open('gpurun_out/r6_bench70.json').read().strip().splitlines()[-1]); print(l['value'], l['ms_per_step'])"
