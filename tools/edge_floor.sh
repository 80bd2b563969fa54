#!/bin/bash
# GPU-box helper: the hand-off edge floor (tools/microbench/edge.hip, built here as tools/edge_floor_bin)
# under first-poll delays: mode 4 = device-wide 1024 granules (8 waves, one pair per lane), mode 5 =
# XCD-local 256 (2 waves); two launches of 2000 rounds per setting
set -o pipefail
for s in 0 1 2 3 4; do
  timeout -k 10 30 ./tools/edge_floor_bin 4 8 2000 $s | tail -2 || exit 1
done
for s in 0 1 2; do
  timeout -k 10 30 ./tools/edge_floor_bin 5 2 2000 $s | tail -2 || exit 1
  timeout -k 10 30 ./tools/edge_floor_bin 5 4 2000 $s | tail -2 || exit 1
done
