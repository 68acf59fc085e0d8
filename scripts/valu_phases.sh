# Dynamic VALU / SALU cost of each phase of the later-bounce kernel (k_bounce<false,false,0>):
# variant libraries that run one phase twice on opaque copies of its inputs (-DPT_DUP=1 closest hit,
# 2 shade, 3 path load); the bench's in-run SQ counters give instructions per segment for each.
# Build (CPU):  VARIANTS="dup1:-DPT_DUP=1 dup2:-DPT_DUP=2 dup3:-DPT_DUP=3" bash scripts/build_variants.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/valu_phases; mkdir -p $O
for v in new ${VS:-dup1 dup2 dup3}; do
  if [ $v = new ]; then unset PT_AMD_LIB; else export PT_AMD_LIB=$R/cuda_pathtracer_amd/build/libpt_amd_$v.so; fi
  timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-scan --no-dropin --pmc-passes 3 \
      > $O/b_$v.json 2> $O/b_$v.err || { echo "bench $v failed"; tail -5 $O/b_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b_$v.json'));r=d['roofline'];u=r.get('valu_issue',{});print('$v', round(d['value'],1), 'valu/seg', round(u.get('instructions_per_segment',0),3), 'salu/launch', u.get('salu_per_launch'), 'segs/launch', r['segments_per_launch'])"
done
