#!/bin/bash
# The persistent launch across processes on one GPU (emulated multi-rank):
# the host-bootstrapped 2-process worker's persist40 / persist80 cases (per-
# iteration time of the persistent launch vs the per-iteration launches of the
# same in-kernel transport, bitwise) and a 1-rank 80^3 line for scale.
# Usage (GPU box): bash tools/persist_multirank.sh  -> gpurun_out/pmr/
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/pmr
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 \
    --master-port 29711 tests/hostcomm_worker.py gpurun_out/pmr > gpurun_out/pmr/worker.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --n 80 --steps 10 --no-secondary --no-cpu-baseline --no-trace-check --no-host-boundary \
    > gpurun_out/pmr/single80.json 2> gpurun_out/pmr/single80.err || exit 1
python3 - <<'PY'
import json
out = {}
for r in (0, 1):
    d = json.load(open(f"gpurun_out/pmr/rank{r}.json"))
    for k in ("persist40", "persist80"):
        c = d[k]
        out[f"{k}_rank{r}"] = {f: c.get(f) for f in ("ok", "used", "same", "retries", "niters",
                                                     "us_per_iter_persistent", "us_per_iter_launches")}
s = json.loads(open("gpurun_out/pmr/single80.json").read().strip().splitlines()[-1])
out["single_rank_80"] = {"value_it_s": s["value"], "us_per_iter": 1e6 / s["value"],
                         "resident_update": s["config"]["options"].get("resident_update")}
json.dump(out, open("gpurun_out/pmr/summary.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
