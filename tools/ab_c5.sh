# interleaved config-5 C3 A/B: product and lib/variants/*.so named on the command line
# (tools/config5.py --fp16 via tools/session.sh; C3 ms of reps 1-3 -> gpurun_out/ab_summary.txt)
set -e
for v in "$@"; do
  if [ $v = product ]; then bash tools/session.sh ab_$v config5; else VARIANT=$v bash tools/session.sh ab_$v config5; fi
  echo "$v $(grep '^rep [123]' gpurun_out/ab_$v/config5.log | awk '{print $7}' | tr '\n' ' ')" >> gpurun_out/ab_summary.txt
done
