# diagnostic: the whole GPU suite with the re-binning's counts memset always queued (variant) and skipped (default)
export TMPDIR=/tmp
O=gpurun_out/${SESSION:-r6dm}; mkdir -p $O
SWRT_LIB_PATH=build/var/memset.so timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/variant.log 2>&1
rc=$?; echo "variant rc=$rc"; tail -5 $O/variant.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/default.log 2>&1
rc=$?; echo "default rc=$rc"; tail -5 $O/default.log
