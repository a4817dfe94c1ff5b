#!/bin/bash
# SQ stall breakdown: x6 pointwise C = 768 on the 16-wave tile and on x6pw, k7 C = 768 for comparison
set -u
export TMPDIR=/tmp
export CONV_PREC=x6 CPMC_NPASS=2
CPMC_DIR=gpurun_out/r05n/pw122 BC_X6_PWDB=0 CONV_ARGS="--cin 768 --cout 768 --k 1 --T 6000 --res --snake --dual" bash tools/lab/conv_pmc.sh || exit 1
CPMC_DIR=gpurun_out/r05n/pwdb BC_X6_PWDB=1 CONV_ARGS="--cin 768 --cout 768 --k 1 --T 6000 --res --snake --dual" bash tools/lab/conv_pmc.sh || exit 1
CPMC_DIR=gpurun_out/r05n/k7 CONV_ARGS="--cin 768 --cout 768 --k 7 --d 3 --T 6000 --snake" bash tools/lab/conv_pmc.sh || exit 1
CPMC_DIR=gpurun_out/r05n/pw192 BC_X6_PWDB=0 CONV_ARGS="--cin 192 --cout 192 --k 1 --T 60000 --res --snake --dual" bash tools/lab/conv_pmc.sh || exit 1
echo done
