# round 6 session d: paper preset (configs[4]) re-anchored at the default precision + the x6 attention's fetch
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
rm -rf gpurun_out/r06d_paper_fetch
RDMI_PROF_SEQ=gpurun_out/r06d_paper_seq.json timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv \
  -d gpurun_out/r06d_paper_fetch -o run -- python3 bench.py --preset paper --frames-total 60 --steps 1 --warmup 0 \
  --no-cpu-baseline --no-validate > gpurun_out/r06d_paper_fetch.log 2>&1 || exit $?
mv gpurun_out/r06d_paper_seq.json gpurun_out/r06d_paper_fetch/seq.json
python tools/traffic_split.py --fetch gpurun_out/r06d_paper_fetch --write gpurun_out/r06d_paper_fetch \
  --family attention_fwd_f32x6 --counters FETCH_SIZE > gpurun_out/r06d_paper_attn_fetch.txt 2>&1
find gpurun_out/r06d_paper_fetch -name '*.csv' -size +20M -delete
timeout -k 10 1000 python -u bench.py --preset paper --steps 1 --warmup 1 --no-cpu-baseline \
  > gpurun_out/r06d_bench_paper.log 2>&1; echo "paper exit $?"
