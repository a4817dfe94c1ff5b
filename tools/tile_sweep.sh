# Tile sweep of the encoder conv shapes (every tile of the chosen precision per shape): profiles/r01_tile_sweep.txt
set -e
mkdir -p gpurun_out
run() { timeout -k 10 300 python tools/conv_bench.py --iters 5 --cfg all --precision ${PRECISION:-h3} "$@" >> gpurun_out/sweep.log 2>&1; }
run --cin 48 --cout 96 --k 4 --s 2 --T 120000 --snake
run --cin 96 --cout 192 --k 4 --s 2 --T 60000 --snake
run --cin 192 --cout 384 --k 4 --s 2 --T 30000 --snake
run --cin 192 --cout 192 --k 7 --d 3 --T 60000 --snake
run --cin 192 --cout 192 --k 1 --T 60000 --res --dual
run --cin 384 --cout 384 --k 7 --d 3 --T 30000 --snake
run --cin 384 --cout 384 --k 1 --T 30000 --res --dual
run --cin 384 --cout 768 --k 10 --s 5 --T 6000 --snake
run --cin 768 --cout 768 --k 7 --d 3 --T 6000 --snake
run --cin 768 --cout 768 --k 1 --T 6000 --res --dual
run --cin 768 --cout 1536 --k 10 --s 5 --T 1200
run --cin 1536 --cout 6144 --k 1 --T 76800 --B 1
run --cin 1536 --cout 1024 --k 3 --T 1200
