#!/bin/bash
# Round 3: stamped timeline of the persistent ResLSTM (h3, H = 1536, T = 1200) at 64 and 32 clips, and the
# work-skipping ablations (BC_LSTM_SEQ_DEBUG 1 no MFMA, 2 no h loads, 4 no flag poll; wrong results).
set -u
mkdir -p gpurun_out
o=gpurun_out/r03q_lstm_stamps.txt; : > $o
for B in 64 32; do
  BC_LSTM_SEQ_STAMPS=1 timeout -k 10 120 python tools/lstm_bench.py --precision h3 --B $B --T 1200 >> $o 2>&1 || { echo "failed B=$B" >> $o; exit 1; }
  for dbg in 1 2 4 6; do
    BC_LSTM_SEQ_DEBUG=$dbg timeout -k 10 120 python tools/lstm_bench.py --precision h3 --B $B --T 1200 >> $o 2>&1 || { echo "failed dbg=$dbg" >> $o; exit 1; }
  done
done
echo done >> $o
