# diagnostic: snapshot kernels with and without their FFT stages (build/var/nofft.so)
export TMPDIR=/tmp
O=gpurun_out/r6snapdiag; mkdir -p $O
for v in def nofft; do
  if [ $v = nofft ]; then export SWRT_LIB_PATH=build/var/nofft.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o s -- python3 tools/owner_legs.py --micro 142857 --receiver --owner --steps 200 > $O/$v.log 2>&1 || exit 1
  echo "== $v"; grep micro $O/$v.log
  python3 - $O/$v <<'PY'
import csv,glob,sys
f=glob.glob(sys.argv[1]+'/**/s_kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'spectra_rows' in r['Name'] or 'cols_pack' in r['Name'] or 'tile_leapfrog' in r['Name']:
        print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,2), round(float(r['MinNs'])/1e3,2))
PY
done
