#!/bin/bash
OUT=gpurun_out/p48
mkdir -p "$OUT"
timeout -k 10 200 python tools/check_plane48.py > "$OUT/check.log" 2>&1
rc=$?; grep -v amdgpu.ids "$OUT/check.log" | tail -4; [ $rc -ne 0 ] && exit $rc
b() { # tag env fabric
  env $2 timeout -k 10 200 python bench.py --fabric $3 --mode shortest --steps ${4:-20} --warmup 2 --no-cpu-baseline > "$OUT/$1.json" 2> "$OUT/$1.err" || { tail -3 "$OUT/$1.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$1.json'));r=d['roofline'];print('$1', 'step %.4f ms'%d['ms_per_step'], 'kernel %.4f ms'%r['kernel_ms'], r['kernel'], 'frac %.3f'%r['frac'])"
}
b k48_dest X=1 fat_tree:48
b k48_plane SDNROUTE_SP_STRATEGY=plane fat_tree:48
b k48_dest2 X=1 fat_tree:48
b k48_plane2 SDNROUTE_SP_STRATEGY=plane fat_tree:48
b torus X=1 torus:32,32,32 3
b jf X=1 jellyfish:100000,16,1 3
b df X=1 dragonfly:16,8,8
