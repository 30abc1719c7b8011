set -e
O=gpurun_out/ablate; mkdir -p $O
for n in A B C D E F G; do echo "== $n" >> $O/log; timeout -k 10 120 tools/build/mb_$n 4096 s 16 >> $O/log 2>&1; done
echo ok
