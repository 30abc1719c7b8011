R=$GRAFT_REPO_ROOT
cd "$R"
for i in 1 2; do
  for cfg in "1 4" "2 4" "1 8" "2 8" "3 4"; do
    set -- $cfg
    NVRX_RB_COPIES=1 NVRX_RB_BPC=$1 NVRX_RB_WAVES=$2 timeout -k 10 120 python tools/ab_zipf.py 10 2>&1 | grep records_stats_ms || exit 1
  done
done
