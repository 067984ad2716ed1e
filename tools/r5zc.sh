set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5zc
for r in 1 2; do for v in base invst; do
  FHECORE_LIB=$PWD/tools/variants/$v.so timeout -k 10 200 python3 tools/time_ntt.py 17 512 >> gpurun_out/r5zc/t.txt 2>/dev/null || exit $?
done; done
echo done
