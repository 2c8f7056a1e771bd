#!/bin/bash
# dist VALU evidence on the GPU box (run via gpurun from the repo root): the
# per-instruction issue rates of the tile kernel's mix (tools/micro/valu_mix)
# and an SQ counter pass over k_snp_tile at N=8192 x L=1 Mbp.
set -o pipefail
TAG=${1:-r02}
R=$PWD
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
echo "== valu_mix" && timeout -k 10 120 $R/tools/micro/valu_mix > $OUT/valu_mix.txt 2>&1 || exit 1
cat $OUT/valu_mix.txt
echo "== pmc SQ (dist)" && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES --output-format csv -d $OUT/pmc_sq_dist -o run -- python3 $R/tools/perf_dist.py 8192 1000000 > $OUT/pmc_sq_dist.log 2>&1 || exit 1
tail -3 $OUT/pmc_sq_dist.log
echo "== done"
echo "== pmc GRBM_GUI_ACTIVE (clock)" && timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc_clk_dist -o run -- python3 $R/tools/perf_dist.py 8192 1000000 > $OUT/pmc_clk_dist.log 2>&1 || exit 1
echo "== done (clock)"
