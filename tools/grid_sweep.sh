# DNJ grid sweep at N=10k (development aid): k_dnj_select / k_dnj_scan grid caps
set -e
for cfg in "1024 2048" "1024 1024" "1024 512" "512 2048" "256 2048" "512 512"; do
  set -- $cfg
  echo "== sel_max $1 scan_max $2"
  CCG_SEL_MAX=$1 CCG_SCAN_MAX=$2 timeout -k 10 120 python tools/quick_perf.py 10000 dnj 2>&1 | grep -E "exact=False|per-kernel" | tail -2
done
