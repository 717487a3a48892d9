#!/bin/bash
# Bench A/B on one box between the in-tree libcvd.so and another build of it
# (e.g. the previous commit's, built in a git worktree and copied here):
#   bash profiles/ab_lib.sh gpurun_out/ab profiles/_old_libcvd.so "m2 r23_m4 m2"
# The other library runs from a copy of the package under $TMPDIR, alternating
# with the in-tree one per config so that box drift hits both.
set -uo pipefail
export TMPDIR=${TMPDIR:-/tmp}
O=$PWD/$1; OLDLIB=$PWD/$2; CONFIGS=${3:-"m2 r23_m4 m2 r23_m4"}
mkdir -p $O
OLD=$TMPDIR/ab_other; rm -rf $OLD; mkdir -p $OLD
cp -r bench.py __graft_entry__.py oracle detecting-convolutional-codes-via-markovian-statistics_amd $OLD/
cp $OLDLIB $OLD/detecting-convolutional-codes-via-markovian-statistics_amd/lib/libcvd.so
show() { python -c "import json;d=json.loads(open('$2').read().strip().splitlines()[-1]);print('$1',d['value'],d['ms_per_step'],'gen',d['diagnostic']['generator_ms_per_step'],'det',d['diagnostic']['detector_ms_per_step'])"; }
i=0
for c in $CONFIGS; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --config $c --cpu-baseline 0 --early-decision 0 > $O/new_${c}_$i.json 2>/dev/null || exit 1
  show "new $c" $O/new_${c}_$i.json
  (cd $OLD && timeout -k 10 300 python bench.py --config $c --cpu-baseline 0 --early-decision 0 > $O/old_${c}_$i.json 2>/dev/null) || exit 1
  show "old $c" $O/old_${c}_$i.json
done
