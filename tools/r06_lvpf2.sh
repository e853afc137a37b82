#!/bin/bash
# Round-6: kernel stats of the config-3 shard per mid-node accumulate variant (alternated),
# only the per-kernel summaries kept
set -o pipefail
OUT=gpurun_out/$1; mkdir -p "$OUT"
export TMPDIR=/tmp
R=$PWD
L=$R/ate_replication_causalml_amd/_lib
cd /tmp
for v in base pf16 u16 pf base pf16 u16 pf; do
  if [ $v = base ]; then unset ATE_HIP_LIB; else export ATE_HIP_LIB=$L/libatehip_$v.so; fi
  D=/tmp/prof_$v
  rm -rf $D
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -- python3 $R/tools/cfg3.py --rows 1e7 --cols 500 --trees 100 --shard 0/8 > $R/$OUT/cfg3_$v.log 2>&1 || exit $?
  f=$(find $D -name '*kernel_stats.csv' | head -1)
  echo "$v: $(tail -1 $R/$OUT/cfg3_$v.log | grep -o '"seconds": [0-9.]*') $(python3 -c "import csv,sys; [print(r['Name'].split('::')[1][:32], r['Calls'], r['TotalDurationNs'], end='; ') for r in csv.DictReader(open(sys.argv[1])) if 'lv_mid' in r['Name'] or 'lv_small' in r['Name']]" $f)"
  cp $f $R/$OUT/kstats_$v.csv
done
