# A/B kernel timing on the GPU: kbench over pipeline variants (env knobs) and the old tree.
mkdir -p gpurun_out
: > gpurun_out/ab.log
for v in "KB_FUSED=0"; do
  echo "== $v" >> gpurun_out/ab.log
  env $v timeout -k 10 240 python tools/kbench.py >> gpurun_out/ab.log 2>&1 || { cat gpurun_out/ab.log; exit 1; }
done
if [ -d build_variants/old ]; then
  echo "== old tree" >> gpurun_out/ab.log
  (cd build_variants/old && timeout -k 10 240 python tools/kbench.py) >> gpurun_out/ab.log 2>&1 || { cat gpurun_out/ab.log; exit 1; }
fi
cat gpurun_out/ab.log
