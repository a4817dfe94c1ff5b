# Wide (x256-column) tiles on the pointwise, strided and LSTM-projection shapes.
set -u
mkdir -p gpurun_out
out=gpurun_out/sweep3.log
run() { timeout -k 10 150 python tools/conv_bench.py --precision h3 --iters 5 "$@" >> $out 2>&1; }
run --cin 384 --cout 384 --k 1 --T 30000 --res --dual --snake --cfg 314,320,321 || exit 1
run --cin 192 --cout 192 --k 1 --T 60000 --res --dual --snake --cfg 314,320 || exit 1
run --cin 768 --cout 768 --k 1 --T 6000 --res --dual --snake --cfg 314,320,321 || exit 1
run --cin 1536 --cout 6144 --k 1 --T 76800 --B 1 --cfg 314,320,321 || exit 1
run --cin 384 --cout 768 --k 10 --s 5 --T 6000 --snake --cfg 302,5320,5321,5300 || exit 1
run --cin 768 --cout 1536 --k 10 --s 5 --T 1200 --cfg 302,5320,5321,5300 || exit 1
run --cin 192 --cout 384 --k 4 --s 2 --T 30000 --snake --cfg 315,2320,2309,2300 || exit 1
run --cin 96 --cout 192 --k 4 --s 2 --T 60000 --snake --cfg 315,2320,2309 || exit 1
run --cin 48 --cout 96 --k 4 --s 2 --T 120000 --snake --cfg 2309,2320 || exit 1
run --cin 1024 --cout 1536 --k 7 --T 1200 --cfg 300,320,321 || exit 1
