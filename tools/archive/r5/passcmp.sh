# the bench's kernel-timing pass vs its timed call in ONE kernel trace: every k_shadow_extend and
# k_walk_resume dispatch in order (timed call = the one before the pass's three calls)
export TMPDIR=/tmp
P=gpurun_out/${1:-r5passcmp}; mkdir -p $P
timeout -s KILL 600 rocprofv3 --kernel-trace -d $P/trace -o k -- python3 bench.py --no-bdpt --no-cpu-baseline --no-roofline-model > $P/bench.json 2> $P/bench.err || { tail -20 $P/bench.err; exit 4; }
python3 - $(find $P/trace -name "*.db" | head -1) <<'PY' | tee $P/dispatches.txt
import sys
sys.path.insert(0, "tools")
from pmc_summary import dispatches
for d in dispatches(sys.argv[1]):
    k = d["kernel"]
    if "k_shadow_extend" in k or "k_walk_resume" in k or "k_primary" in k:
        print(("k_shadow_extend" if "k_shadow_extend" in k else "k_walk_resume" if "k_walk_resume" in k else "k_primary"), d["grid"], round(d["ms"], 4))
PY
python3 tools/bench_summary.py $P/bench.json
find $P/trace -name "*.db" -delete
