# Workgroup order experiment: m-tile innermost (default) vs outermost (BC_X6_DEBUG=32)
set -u
mkdir -p gpurun_out
for dbg in 0 32; do
  echo "== dbg $dbg" >> gpurun_out/mmajor.log
  run() { BC_X6_DEBUG=$dbg timeout -k 10 150 python tools/conv_bench.py --precision h3 --iters 5 "$@" >> gpurun_out/mmajor.log 2>&1; }
  run --cin 384 --cout 384 --k 7 --d 3 --T 30000 --snake --cfg 320 || exit 1
  run --cin 768 --cout 768 --k 7 --d 3 --T 6000 --snake --cfg 321 || exit 1
  run --cin 192 --cout 192 --k 7 --d 3 --T 60000 --snake --cfg 320 || exit 1
  run --cin 384 --cout 384 --k 1 --T 30000 --res --dual --snake --cfg 314 || exit 1
  run --cin 768 --cout 768 --k 1 --T 6000 --res --dual --snake --cfg 314 || exit 1
  run --cin 384 --cout 768 --k 10 --s 5 --T 6000 --snake --cfg 5321 || exit 1
  run --cin 768 --cout 1536 --k 10 --s 5 --T 1200 --cfg 5321 || exit 1
  run --cin 1536 --cout 6144 --k 1 --T 76800 --B 1 --cfg 321 || exit 1
  run --cin 192 --cout 384 --k 4 --s 2 --T 30000 --snake --cfg 315 || exit 1
done
