set -u
bash tools/gpu_session.sh r03p tests || exit $?
for rep in 1 2; do
  timeout -k 10 300 python bench.py --config cfg5 --steps 10 --warmup 2 --no-cpu --no-e2e > gpurun_out/r03p/cfg5_$rep.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r03p/cfg5_$rep.log') if l.startswith('{')][0]); print('cfg5', d['ms_per_step'], d['kernels'], d['parity_checked_frames']['pass'], d['parity_checked_frames']['max_abs_ddb_within_100dB'])"
done
V=pypanadapter_amd/lib/variants
AB_REPS=2 bash tools/ab.sh r03p_ab base=default p5w3=$V/libzfft_p5w3.so p2w3=$V/libzfft_p2w3.so
AB_ARGS="--frames 6144" AB_REPS=2 bash tools/ab.sh r03p_ab6k base=default p5w3=$V/libzfft_p5w3.so p2w3=$V/libzfft_p2w3.so
