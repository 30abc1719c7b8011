#!/bin/bash
# A/B of record-bucketing block shapes on configs[3] (tools/ab_zipf.py).
for w in 4 16; do for b in 0 1 2; do
  echo -n "waves=$w bpc=$b: "; NVRX_RB_WAVES=$w NVRX_RB_BPC=$b timeout -k 10 200 python tools/ab_zipf.py 4 2>/dev/null | tail -1
done; done
