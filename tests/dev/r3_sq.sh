# SQ instruction counters of the pair and one-pod resolvers (tests/dev/ab_pair.py workload).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
ROOT=$(pwd)
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d /tmp/sq -o run -- python3 $ROOT/tests/dev/ab_pair.py > $ROOT/gpurun_out/sq_ab.txt 2>&1 || exit 1
cd $ROOT
python3 - <<'PY'
import sys, json
sys.path.insert(0, "profiles")
from db_summary import per_kernel
d = per_kernel("/tmp/sq/run_results.db")
out = {k: {c: round(v[0], 1) for c, v in cs.items()} for k, cs in d.items() if "resolve" in k}
print(json.dumps(out, indent=1))
json.dump(out, open("gpurun_out/sq_resolvers.json", "w"), indent=1)
PY
