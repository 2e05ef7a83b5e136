#!/bin/bash
# full GPU parity, then profiles of the k=48 shortest (bit-plane BFS) and APSP
# (64-tile) lines and the torus / dragonfly shortest lines (balanced chunks)
set -u
OUT=gpurun_out/r2g
mkdir -p "$OUT" gpurun_out/sum
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_gpu.log"; [ $rc -ne 0 ] && exit $rc
for f in fat_tree:48 torus:32,32,32 dragonfly:16,8,8; do
  timeout -k 10 200 python bench.py --fabric $f --mode shortest --steps 10 --warmup 2 --no-cpu-baseline \
    > "$OUT/sp_$f.json" 2> "$OUT/sp_$f.err" || exit 1
  python -c "import json;d=json.load(open('$OUT/sp_$f.json'));r=d['roofline'];print('$f', 'step %.4f ms'%d['ms_per_step'], 'kernel %.4f ms'%r['kernel_ms'], r['kernel'], 'frac %.3f'%r['frac'])"
done
P() {
  local tag=$1; shift
  bash tools/profile_gpu.sh "$tag" "$@" > /dev/null || exit $?
  python3 tools/summarize_profile.py "gpurun_out/prof_$tag" "gpurun_out/sum/$tag" > /dev/null || exit 1
  rm -rf "gpurun_out/prof_$tag"
  echo "profiled $tag"
}
P r02_sp48 --mode shortest
P r02_apsp48 --mode apsp --steps 5 --warmup 1
P r02_torus_sp --fabric torus:32,32,32 --mode shortest --steps 2 --warmup 1
P r02_df_sp --fabric dragonfly:16,8,8 --mode shortest
exit 0
