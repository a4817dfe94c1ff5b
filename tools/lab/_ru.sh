mkdir -p gpurun_out
for c in 0 109 104 106; do
  echo "== BC_RU_CFG=$c" >> gpurun_out/ru.log
  BC_RU_CFG=$c timeout -k 10 200 python tools/layer_profile.py 2>&1 | grep -E "step|resunit|k=7 s=1 d=[139] T=(120000|240000)|k=1 s=1 d=1 T=(120000|240000)" >> gpurun_out/ru.log || exit 1
done
