#!/bin/bash
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
for w in 8 4 2 1; do echo "wps=$w" >> $OUT/ub.txt; timeout -k 10 60 ./tools/ubench_fnv.bin $w | grep "rep 2" >> $OUT/ub.txt; done
