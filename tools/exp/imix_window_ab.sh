cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/imix
cp halo_amd/lib/libhalo_rx.so /tmp/orig.so
for v in w256 w128 w64; do
  cp tools/exp/libhalo_rx_$v.so halo_amd/lib/libhalo_rx.so
  timeout -k 10 120 python tools/tune.py --only imix > gpurun_out/imix/tune_$v.log 2>&1 || break
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/imix/f_$v -o run -- python3 tools/prof_kernels.py config3_imix_16M > gpurun_out/imix/f_$v.log 2>&1 || break
done
cp /tmp/orig.so halo_amd/lib/libhalo_rx.so
grep -h 'imix' gpurun_out/imix/tune_*.log
