#!/bin/bash
# One GPU-box session: each GPU step under its own time limit; stop at the first crash,
# abort, fault or timeout (pytest's "tests failed" exit code 1 does not stop the session).
# Usage: bash tools/gpu_session.sh <tag> [steps...]   steps: test smoke bench prof pmc
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
step() {
  local name=$1 limit=$2; shift 2
  echo "[$(date +%T)] start $name" | tee -a "$OUT/steps.log"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    test)  step pytest_gpu 1200 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread ;;
    tlo)   step pytest_lo 600 python -u -m pytest tests/test_gpu_loopback.py tests/test_gpu_tx_build.py -m gpu -q -rf -x --timeout 120 --timeout-method thread ;;
    ttx)   step pytest_tx 600 python -m pytest tests/test_gpu_tx.py -m gpu -q -rf -x ;;
    thash) step pytest_hash 600 python -m pytest tests/test_gpu_flow_hash.py -m gpu -q -rf -x ;;
    troute) step pytest_route 600 python -m pytest tests/test_gpu_route.py -m gpu -q -rf -x ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 900 python bench.py ;;
    benchq) step benchq 600 python bench.py --no-secondary --cpu-seconds 4 ;;
    prof)  step prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --no-cpu --steps 20 ;;
    pmcf)  step pmc_fetch 900 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 bench.py --no-cpu --steps 10 --warmup 2 ;;
    pmcw)  step pmc_write 900 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 bench.py --no-cpu --steps 10 --warmup 2 ;;
    tune)  step tune 900 python tools/tune.py ;;
    dist2) step dist2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 50 --warmup 5 ;;
    list)  step counters 300 rocprofv3 -L ;;
    kt)    step kt 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 tools/prof_kernels.py ${PK_ARGS:-} ;;
    kfetch) step kfetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/kfetch" -o run -- python3 tools/prof_kernels.py ${PK_ARGS:-} ;;
    kwrite) step kwrite 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/kwrite" -o run -- python3 tools/prof_kernels.py ${PK_ARGS:-} ;;
    ksq)   step ksq 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$OUT/ksq" -o run -- python3 tools/prof_kernels.py ${PK_ARGS:-} ;;
    tuneq) step tuneq 600 python tools/tune.py --quick ;;
    tstream) step pytest_stream 600 python -u -m pytest tests/test_gpu_stream.py -m gpu -q -rf -x --timeout 120 --timeout-method thread ;;
    gpus2) step gpus2 600 python bench.py --gpus 2 --steps 50 --warmup 5 --no-secondary --no-cpu ;;
    tunes) step tune_stream 600 python tools/tune.py --spec imix:-2,570B:-2,128B:-2,1500B:8 ;;
    ringn) step ring_native 600 python tools/bench_ring_native.py --sweep ;;
    ringprof) step ring_prof 600 rocprofv3 --kernel-trace --hip-runtime-trace --stats --output-format csv -d "$OUT/ringprof" -o run -- python3 tools/bench_ring_native.py --iters 500 ${RP_ARGS:-} ;;
    tunev) step tune_variants 600 python tools/tune.py --only 570B,1500B,jumbo9000,imix --variants 4,8,16,-3,-2,-1 ;;
    abold) step ab_old_new 900 bash tools/exp/ab_variants.sh "python tools/tune.py --spec 1500B:8,570B:4,jumbo9000:16,imix:-1,64B:1" old new ;;
    abtx) step ab_tx 900 bash tools/exp/ab_variants.sh "python tools/exp/bench_tx.py && python tools/exp/bench_tx_build.py" old new ;;
    ttxall) step pytest_txall 600 python -u -m pytest tests/test_gpu_tx.py tests/test_gpu_tx_build.py -m gpu -q -rf -x --timeout 120 --timeout-method thread ;;
    abtxs) step ab_tx_store 900 bash tools/exp/ab_variants.sh "python tools/exp/bench_tx.py" txa txfull txnt txfullnt ;;
    kwrq)  step kwrq 300 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d "$OUT/kwrq" -o run -- python3 tools/exp/bench_tx.py ;;
    ptxb)  step probe_txb 300 ./tools/exp/probe_txb ;;
    tring) step pytest_ring 600 python -u -m pytest tests/test_gpu_ring.py -m gpu -q -rf -x --timeout 120 --timeout-method thread ;;
    abtx3) step ab_tx3 900 bash tools/exp/ab_variants.sh "python tools/exp/bench_tx.py && python tools/exp/bench_tx_build.py" txg1 txg4 txbnew ;;
    kgap)  step kgap 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/kgap" -o run -- python3 tools/exp/gap_fetch.py ;;
    absvc) step ab_svc 900 bash tools/exp/ab_variants.sh "python tools/bench_ring_native.py --persistent --frames 1 --iters 3000 && python tools/bench_ring_native.py --persistent --frames 1000 --iters 3000" ${AB_SVC:-svcA svcB} ;;
    krd)   step krd 600 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum --output-format csv -d "$OUT/krd" -o run -- python3 tools/prof_kernels.py ${PK_ARGS:-} ;;
    kwrq2) step kwrq2 600 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d "$OUT/kwrq" -o run -- python3 tools/prof_kernels.py ${PK_ARGS:-} ;;
    krdgap) step krdgap 300 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum --output-format csv -d "$OUT/krdgap" -o run -- python3 tools/exp/gap_fetch.py ;;
    abtxc) step ab_txc 900 bash tools/exp/ab_variants.sh "python tools/exp/bench_tx.py" txc0 txc1 txc2 ;;
    abtail) step ab_tail 900 bash tools/exp/ab_variants.sh "python tools/tune.py --spec 1500B:8,570B:4,imix:-1,imix:-2,jumbo9000:16" tl0 tl1 ;;
    vtail) step vtail 600 bash tools/exp/variant_tests.sh "tests/test_gpu_parity.py tests/test_gpu_stream.py -m gpu" tl1 ;;
    krdtail) step krdtail 600 bash tools/exp/with_variant.sh tl1 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum --output-format csv -d "$OUT/krdtail" -o run -- python3 tools/prof_kernels.py 1500B_udp_1M ;;
    krdr12) step krdr12 600 bash tools/exp/with_variant.sh r12 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum --output-format csv -d "$OUT/krdr12" -o run -- python3 tools/prof_kernels.py 1500B_udp_1M ;;
    plines) step plines 300 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum --output-format csv -d "$OUT/plines" -o run -- ./tools/exp/probe_lines ;;
    abtail2) step ab_tail2 900 bash tools/exp/ab_variants.sh "python tools/tune.py --spec 1500B:8,570B:4,jumbo9000:16,imix:-1" tl0 tl2 ;;
    vtail2) step vtail2 600 bash tools/exp/variant_tests.sh "tests/test_gpu_parity.py tests/test_gpu_stream.py -m gpu" tl2 ;;
    krdtail2) step krdtail2 600 bash tools/exp/with_variant.sh tl2 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum --output-format csv -d "$OUT/krdtail2" -o run -- python3 tools/prof_kernels.py 1500B_udp_1M ;;
    abov) step ab_ov 900 bash tools/exp/ab_variants.sh "python tools/tune.py --spec 1500B:8,570B:4,jumbo9000:16,imix:-1,imix:-2,64B:1" tl0 ov1 ;;
    vov) step vov 600 bash tools/exp/variant_tests.sh "tests/test_gpu_parity.py tests/test_gpu_stream.py tests/test_gpu_tx.py -m gpu" ov1 ;;
    krdov) step krdov 600 bash tools/exp/with_variant.sh ov1 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum --output-format csv -d "$OUT/krdov" -o run -- python3 tools/prof_kernels.py 1500B_udp_1M config3_imix_16M ;;
    abnt) step ab_nt 900 bash tools/exp/ab_variants.sh "python tools/tune.py --spec 1500B:8,570B:4,jumbo9000:16,imix:-1" tl0 nt1 nt2 ;;
    krdnt) step krdnt 600 bash -c "bash tools/exp/with_variant.sh nt1 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum --output-format csv -d $OUT/krdnt1 -o run -- python3 tools/prof_kernels.py 1500B_udp_1M && bash tools/exp/with_variant.sh nt2 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum --output-format csv -d $OUT/krdnt2 -o run -- python3 tools/prof_kernels.py 1500B_udp_1M" ;;
    abxx) step ab_xxh3 900 bash tools/exp/ab_variants.sh "python tools/exp/bench_xxh3.py" ${AB_XX:-xx8 xx4} ;;
    abg8) step ab_g8 900 bash tools/exp/ab_variants.sh "python tools/tune.py --spec 1500B:8,imix:-1,570B:8" ${AB_G8:-g8shfl g8dpp} ;;
    ktxx)  step ktxx 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ktxx" -o run -- python3 tools/exp/bench_xxh3.py ;;
    sqxx)  step sqxx 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$OUT/sqxx" -o run -- python3 tools/exp/bench_xxh3.py ;;
    rdxx)  step rdxx 300 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum --output-format csv -d "$OUT/rdxx" -o run -- python3 tools/exp/bench_xxh3.py ;;
    abgen) step ${AB_NAME:-ab_gen} 900 bash tools/exp/ab_variants.sh "$AB_CMD" $AB_V ;;
    krdv)  step krd_$KV 600 bash tools/exp/with_variant.sh $KV rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum --output-format csv -d "$OUT/krd_$KV" -o run -- python3 tools/prof_kernels.py ${PK_ARGS:-} ;;
    wrxx)  step wrxx 300 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d "$OUT/wrxx" -o run -- python3 tools/exp/bench_xxh3.py ;;
    vgen)  step vtest_$VT 600 bash tools/exp/variant_tests.sh "$VT_TESTS" $VT ;;
    tres)  step pytest_resident 600 python -u -m pytest tests/test_gpu_host_resident.py tests/test_gpu_ring.py tests/test_gpu_single_frame.py tests/test_gpu_engine_cadence.py -m gpu -q -rf -x --timeout 120 --timeout-method thread ;;
    dropin) step dropin 600 python tools/bench_dropin.py ;;
    tmulti) step pytest_multi 600 python -u -m pytest tests/test_gpu_multi_batch.py -m gpu -q -rf -x --timeout 120 --timeout-method thread ;;
    tnew)  step pytest_new 900 python -u -m pytest tests/test_gpu_host_resident.py tests/test_gpu_multi_batch.py tests/test_gpu_ring.py tests/test_gpu_single_frame.py tests/test_gpu_engine_cadence.py tests/test_gpu_route.py -m gpu -q -rf -x --timeout 120 --timeout-method thread ;;
    ttxb)  step pytest_txb 600 python -u -m pytest tests/test_gpu_tx_build.py tests/test_gpu_loopback.py -m gpu -q -rf -x --timeout 120 --timeout-method thread ;;
    thist) step pytest_hist 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi_batch.py -k "histogram or hist or multi" -m gpu -q -rf -x --timeout 120 --timeout-method thread ;;
    abxb)  step ab_xxh3_bf 900 bash tools/exp/ab_variants.sh "python tools/exp/bench_xxh3.py" ${AB_XB:-xxbf0 new} ;;
    abtp)  step ab_tx_pipe 900 bash tools/exp/ab_variants.sh "python tools/exp/bench_tx_build.py" ${AB_TP:-txpipe0 new} ;;
    vtx)   step vtx 600 bash tools/exp/variant_tests.sh "tests/test_gpu_tx_build.py tests/test_gpu_loopback.py -m gpu" ${VT:-txbu} ;;
    vxx)   step vxx 600 bash tools/exp/variant_tests.sh "tests/test_gpu_flow_hash.py -m gpu" ${VX:-xxg8} ;;
    txlay) step tx_layout 600 python tools/exp/tx_layout_sweep.py ;;
    txx)   step pytest_xxh3 600 python -u -m pytest tests/test_gpu_flow_hash.py -m gpu -q -rf -x --timeout 120 --timeout-method thread ;;
    prof4) PK_ARGS="${PK4:-config2 config2_batch_stream lo_drain_1M_50B flow_hash_config2 flow_hash_config2_compact tx_build_udp_256k_1514B}"
           step kt 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 tools/prof_kernels.py $PK_ARGS
           step krd 600 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum --output-format csv -d "$OUT/krd" -o run -- python3 tools/prof_kernels.py $PK_ARGS
           step kwrq 600 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d "$OUT/kwrq" -o run -- python3 tools/prof_kernels.py $PK_ARGS
           step ksq 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$OUT/ksq" -o run -- python3 tools/prof_kernels.py $PK_ARGS ;;
    txbc)  PK_ARGS="tx_build_udp_1M_64B tx_build_udp_256k_1514B probe_tx_build_64B probe_tx_build_1514B"
           step txb_kt 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/txb_kt" -o run -- python3 tools/prof_kernels.py $PK_ARGS
           step txb_sq1 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$OUT/txb_sq1" -o run -- python3 tools/prof_kernels.py $PK_ARGS
           step txb_sq2 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH --output-format csv -d "$OUT/txb_sq2" -o run -- python3 tools/prof_kernels.py $PK_ARGS
           step txb_rd 300 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum --output-format csv -d "$OUT/txb_rd" -o run -- python3 tools/prof_kernels.py $PK_ARGS
           step txb_wr 300 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d "$OUT/txb_wr" -o run -- python3 tools/prof_kernels.py $PK_ARGS ;;
    pshape) step probe_shapes 300 python tools/exp/probe_shapes.py ;;
    profhead) step profhead 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profhead" -o run -- python3 bench.py --no-secondary --no-cpu ;;
    timix) step tune_imix 300 python tools/tune.py --spec imix:0,570B:0 && step tune_imix2 300 python tools/tune.py --spec imix:-2,570B:-2 ;;
    pmcall) PK_ARGS="${PKALL:-}"
           step kt 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 tools/prof_kernels.py $PK_ARGS
           step kfetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/kfetch" -o run -- python3 tools/prof_kernels.py $PK_ARGS
           step kwrite 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/kwrite" -o run -- python3 tools/prof_kernels.py $PK_ARGS
           step krd 600 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum --output-format csv -d "$OUT/krd" -o run -- python3 tools/prof_kernels.py $PK_ARGS
           step kwrq 600 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d "$OUT/kwrq" -o run -- python3 tools/prof_kernels.py $PK_ARGS
           step ksq 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$OUT/ksq" -o run -- python3 tools/prof_kernels.py $PK_ARGS ;;
    *) echo "unknown step $s" ;;
  esac
done
echo done
