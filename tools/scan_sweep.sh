set -e
for cfg in "16 1024" "4 2048" "2 4096" "8 2048"; do
  set -- $cfg
  echo "== div $1 max $2"
  CCG_SCAN_DIV=$1 CCG_SCAN_MAX=$2 timeout -k 10 300 python tools/c3_prof.py 8000 1000000 2>&1 | grep -E "md5|exact=False|dnj_scan|update" | head -4
  CCG_SCAN_DIV=$1 CCG_SCAN_MAX=$2 timeout -k 10 200 python tools/quick_perf.py 2>&1 | grep -E "dnj exact=False"
done
