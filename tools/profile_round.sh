#!/bin/bash
# Round profile on the GPU box (run via gpurun from the repo root):
#   bench line, kernel-trace stats, FETCH_SIZE and WRITE_SIZE PMC passes (one
#   counter group per pass, no trace domains) of the exact-sum DNJ and NJ runs,
#   a PMC calibration pass on a kernel with a known byte count, the VALU issue
#   rates of the dist instruction mix (tools/micro/valu_mix) and an SQ counter
#   pass on the dist tile kernel.  Outputs under gpurun_out/prof_<tag>/.
set -o pipefail
TAG=${1:-r02}
R=$PWD
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
echo "== bench" && timeout -k 10 600 python3 $R/bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
tail -c 400 $OUT/bench.json
echo "== kernel trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-extras --no-cpu > $OUT/trace.log 2>&1 || exit 1
echo "== pmc FETCH_SIZE" && timeout -k 10 420 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/tools/perf_dnj.py 10000 dnj exact > $OUT/pmc_fetch.log 2>&1 || exit 1
echo "== pmc WRITE_SIZE" && timeout -k 10 420 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $R/tools/perf_dnj.py 10000 dnj exact > $OUT/pmc_write.log 2>&1 || exit 1
echo "== pmc FETCH_SIZE nj" && timeout -k 10 420 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_nj -o run -- python3 $R/tools/perf_dnj.py 10000 nj exact > $OUT/pmc_fetch_nj.log 2>&1 || exit 1
echo "== pmc WRITE_SIZE nj" && timeout -k 10 420 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write_nj -o run -- python3 $R/tools/perf_dnj.py 10000 nj exact > $OUT/pmc_write_nj.log 2>&1 || exit 1
echo "== pmc calibration" && timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_cal -o run -- $R/tools/micro/rescan > $OUT/pmc_cal.log 2>&1 || exit 1
echo "== done"; ls -R $OUT | head -40
