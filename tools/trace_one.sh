#!/bin/bash
# kernel trace of dfl001 HSD solves (developer tool): per-kernel stats and the
# k_tail_pr step durations summarised on the box (the database stays there)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-t1}
mkdir -p gpurun_out/prof_$tag
IPO_HIP_DEBUG_REDO=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_trace -o run -- python3 tools/exit_probe.py plain dfl001 2 > gpurun_out/${tag}_trace.log 2>&1 || exit 1
python3 - "$tag" <<'PY' || exit 1
import json, sqlite3, sys
tag = sys.argv[1]
c = sqlite3.connect(f"gpurun_out/{tag}_trace/run_results.db")
rows = list(c.execute("select name, total_calls, total_duration, average from top_kernels order by total_duration desc limit 25"))
steps = [round((e - b) / 1000.0, 1) for b, e in c.execute("select start, end from kernels where name like '%k_tail_pr%' order by start limit 700")]
json.dump({"top": rows, "k_tail_pr": steps}, open(f"gpurun_out/prof_{tag}/summary.json", "w"))
PY
rm -rf gpurun_out/${tag}_trace
