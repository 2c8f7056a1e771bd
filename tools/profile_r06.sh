#!/bin/bash
# Round-6 profiles (run on the GPU box from the repo root):
#   h:  the headline step (configs[2] dist + exact DNJ, the pipelined form
#       bench.py times): kernel trace + stats; then FETCH_SIZE and WRITE_SIZE
#       in separate PMC passes over the sequential form (counter collection
#       serialises the kernels anyway; bytes per launch are the same);
#   clk: the dist kernel's clock and issue counters on the sequential form
#       (GRBM_GUI_ACTIVE against the kernel's duration gives the clock the
#       chip held; SQ_BUSY_CYCLES, SQ_INSTS_VALU / _MFMA the issue mix);
#   c1: configs[1] (10k DNJ exact) kernel trace + FETCH/WRITE passes.
# The per-dispatch CSVs are summarised on the box and removed (a 50k-join
# tree's are too big to ship); summaries go to profiles/.
# Each pass is its own bounded process; a pass that fails ends the script.
set -e
export TMPDIR=/tmp
O=gpurun_out/prof_r06
mkdir -p $O
trap 'rc=$?; echo "exit $rc"; rm -rf $O/*/run_kernel_trace.csv $O/*/run_counter_collection.csv $O/*/*.db $O/*/*/' EXIT
H="python3 bench.py --steps 1 --warmup 0 --no-extras --no-cpu"
HP="python3 bench.py --steps 1 --warmup 0 --no-extras --no-cpu --tree-cus 0"
for part in "$@"; do
  case $part in
  h)
    echo "headline trace"
    timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_h -o run -- $H > $O/trace_h.log 2>&1
    echo "headline FETCH_SIZE"
    timeout -k 10 420 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_h -o run -- $HP > $O/pmc_fetch_h.log 2>&1
    echo "headline WRITE_SIZE"
    timeout -k 10 420 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_h -o run -- $HP > $O/pmc_write_h.log 2>&1
    python3 tools/pmc_summary.py --symbols $O $O/pmc_headline.json "python3 bench.py --steps 1 --warmup 0 --no-extras --no-cpu --tree-cus 0 (configs[2]: 50k x 5M dist + exact DNJ, sequential form)" > /dev/null
    echo "headline summarised"
    ;;
  clk)
    echo "dist clock / issue counters"
    timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $O/pmc_clk -o run -- python3 tools/perf_dist.py 50000 5000000 > $O/pmc_clk.log 2>&1
    python3 tools/pmc_clock.py $O/pmc_clk $O/pmc_clk.json > /dev/null
    echo "clock summarised"
    ;;
  c1)
    echo "configs[1] trace"
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c1 -o run -- python3 tools/perf_dnj.py 10000 dnj exact > $O/trace_c1.log 2>&1
    for c in FETCH_SIZE WRITE_SIZE; do
      lc=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
      echo "configs[1] $c"
      timeout -k 10 200 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$lc -o run -- python3 tools/perf_dnj.py 10000 dnj exact > $O/pmc_$lc.log 2>&1
    done
    python3 tools/pmc_summary.py $O $O/pmc_c1.json > /dev/null
    echo "configs[1] summarised"
    ;;
  esac
done
