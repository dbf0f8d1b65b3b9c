set -e
mkdir -p gpurun_out
for sb in 8 16; do for vb in 8 16; do
  echo "== snippet_batch=$sb vae_batch=$vb" >> gpurun_out/abl.log
  timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --snippet-batch $sb --vae-batch $vb 2>&1 | grep metric | cut -c1-220 >> gpurun_out/abl.log
done; done
