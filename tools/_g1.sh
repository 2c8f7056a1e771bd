set -o pipefail
timeout -k 10 400 python tools/sweep_dnj.py 10000 "" "CCG_PLAN_REGSEL=0" "CCG_PLAN_FR=8" "CCG_PLAN_FR=4" "CCG_PLAN_FR=2" "CCG_PLAN_FR=1" > gpurun_out/g1_sweep.log 2>&1 &&
timeout -k 10 200 python -u -m pytest tests/test_gpu_large.py -x -q --timeout 250 --timeout-method thread -k "config1_dnj" > gpurun_out/g1_tests.log 2>&1
