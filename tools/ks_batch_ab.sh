cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/s3
for r in 1 2; do for b in 16 32 64; do
  timeout -k 10 150 python3 bench.py --workload keyswitch --no-cpu-baseline --ks-batch $b > gpurun_out/s3/ks_b${b}_${r}.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/s3/ks_b${b}_${r}.json')); print($b, d['value'], d['ms_per_step'], d['kernel_ms'])" | tee -a gpurun_out/s3/ksb.txt
done; done
