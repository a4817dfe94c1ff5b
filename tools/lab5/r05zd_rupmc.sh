#!/bin/bash
# SQ counters of the x6 C = 48 and C = 96 ResidualUnits (the encoder flow: snake on load, dual output)
set -u
export TMPDIR=/tmp
RU_PREC=x6 RPMC_DIR=gpurun_out/r05zd/ru48 RU_ARGS="--C 48 --d 3 --T 240000 --lazy --dual" bash tools/lab/ru_pmc.sh || exit 1
RU_PREC=x6 RPMC_DIR=gpurun_out/r05zd/ru96 RU_ARGS="--C 96 --d 3 --T 120000 --lazy --dual" bash tools/lab/ru_pmc.sh || exit 1
echo done
