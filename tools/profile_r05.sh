#!/bin/bash
# Round-5 profiles (run on the GPU box from the repo root):
#   headline step (configs[2] dist + exact DNJ, the pipelined form bench.py
#   times: dist beside tree on disjoint CUs): kernel trace + stats, then
#   FETCH_SIZE and WRITE_SIZE in separate PMC passes (sequential form: counter
#   collection serialises the kernels anyway; bytes per launch are the same);
#   configs[1] (10k DNJ
#   exact) the same.  The per-dispatch CSVs are summarised on the box and
#   removed (a 50k-join tree's are too big to ship); summaries go to profiles/.
set -e
export TMPDIR=/tmp
export CCG_BENCH_CLEAN_EXIT=1   # bench.py's normal exit: rocprofv3 writes its files at exit
O=gpurun_out/prof_r05
mkdir -p $O
trap 'rc=$?; echo "exit $rc"; rm -rf $O/*/run_kernel_trace.csv $O/*/run_counter_collection.csv $O/*/*.db $O/*/*/' EXIT
H="python3 bench.py --steps 1 --warmup 0 --no-extras --no-cpu"
HP="python3 bench.py --steps 1 --warmup 0 --no-extras --no-cpu --tree-cus 0"
if [ "$1" != "c1" ]; then
  echo "headline trace"
  timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_h -o run -- $H > $O/trace_h.log 2>&1
  echo "headline FETCH_SIZE"
  timeout -k 10 420 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_h -o run -- $HP > $O/pmc_fetch_h.log 2>&1
  echo "headline WRITE_SIZE"
  timeout -k 10 420 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_h -o run -- $HP > $O/pmc_write_h.log 2>&1
  python3 tools/pmc_summary.py --symbols $O $O/pmc_headline.json "python3 bench.py --steps 1 --warmup 0 --no-extras --no-cpu (configs[2]: 50k x 5M dist + exact DNJ)" > /dev/null
  echo "headline summarised"
fi
if [ "$1" != "h" ]; then
  echo "configs[1] trace"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c1 -o run -- python3 tools/perf_dnj.py 10000 dnj exact > $O/trace_c1.log 2>&1
  for c in FETCH_SIZE WRITE_SIZE; do
    lc=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
    echo "configs[1] $c"
    timeout -k 10 200 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$lc -o run -- python3 tools/perf_dnj.py 10000 dnj exact > $O/pmc_$lc.log 2>&1
  done
  python3 tools/pmc_summary.py $O $O/pmc_c1.json > /dev/null
  echo "configs[1] summarised"
fi
