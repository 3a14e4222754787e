# nontemporal hints, more streams: the GRM slab reduce and the exact GRM transpose, the default build (hints on)
# against plain-load builds (tools/build_nt_variants.sh: red_plain, C2 step stages; xtp_plain, rocprofv3 kernel
# stats of the exact GRM stage)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ntm
mkdir -p $O
for r in 1 2; do
  for v in default red_plain; do
    if [ $v = default ]; then L=genomicbreedingmodels.jl_amd/gbm/libgbm.so; else L=variants/libgbm_$v.so; fi
    GBM_LIBGBM=$L timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cpu-c3 --no-host-path --no-exact \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['ms_per_step'],3), {k: round(v,4) for k, v in d['stage_ms'].items()})" >> $O/red.txt
  done
done
for v in default xtp_plain default xtp_plain; do
  if [ $v = default ]; then L=$GRAFT_REPO_ROOT/genomicbreedingmodels.jl_amd/gbm/libgbm.so; else L=$GRAFT_REPO_ROOT/variants/libgbm_$v.so; fi
  rm -rf /tmp/ntm_$v
  GBM_LIBGBM=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ntm_$v -o run -- python3 $GRAFT_REPO_ROOT/tools/time_grm_exact.py > /dev/null 2>&1
  python3 -c "
import csv,glob
f=glob.glob('/tmp/ntm_$v/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'xg_' in r['Name']: print('$v', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
" >> $O/xtp.txt
done
GBM_LIBGBM=$GRAFT_REPO_ROOT/variants/libgbm_xtp_plain.so timeout -k 10 200 python3 tools/exact_digest.py >> $O/xtp.txt 2>/dev/null
