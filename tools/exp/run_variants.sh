#!/bin/bash
# A/B of tools/exp/_var/* builds: rounds of every variant in turn, one process per run
# usage: run_variants.sh <out dir> <rounds> <tool.py> [tool args]
set -e
O=$1; ROUNDS=$2; TOOL=$3; shift 3
mkdir -p $O
for r in $(seq $ROUNDS); do
  for v in $(ls tools/exp/_var | grep -v '\.o$'); do
    timeout -k 10 120 python tools/exp/variants.py run $v -- $TOOL "$@" | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/variants.jsonl
  done
done
echo done
