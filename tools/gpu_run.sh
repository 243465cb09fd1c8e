#!/bin/bash
# One evidence pass on a GPU box (run through gpurun from the repo root):
#   bash tools/gpu_run.sh <outdir> [steps...]
# steps (default: tests smoke bench): tests | smoke | bench | distbench | rehearse2 | py:<script>[:args] | kprof | seqprof | pmc | insitu | attr | batch:<B> | probe:<tools binary>
#   | gpuonly:<pytest -k expr, + for spaces> | vtests:<variant>:<expr> | ab:<variant>[,<variant>...] (tools/variants/<name>/libvo.so)
# Every GPU step has its own time limit and the chain stops at the first failure.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:?outdir}; shift; mkdir -p $O
STEPS=${@:-tests smoke bench}
for st in $STEPS; do
  case $st in
  tests)
    timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 \
      || { tail -40 $O/gpu_tests.log; exit 1; }
    tail -1 $O/gpu_tests.log ;;
  gpuonly:*)
    k=${st#gpuonly:}; timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "${k//+/ }" > $O/gpu_sel.log 2>&1 \
      || { tail -40 $O/gpu_sel.log; exit 1; }
    tail -1 $O/gpu_sel.log ;;
  vtests:*)
    # vtests:<variant>:<pytest -k expr, + for spaces> — GPU tests against tools/variants/<variant>/libvo.so
    a=${st#vtests:}; v=${a%%:*}; k=${a#*:}
    VO_LIBPATH=$PWD/tools/variants/$v/libvo.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "${k//+/ }" > $O/vtests_$v.log 2>&1 \
      || { tail -40 $O/vtests_$v.log; exit 1; }
    tail -1 $O/vtests_$v.log ;;
  smoke)
    timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
    tail -1 $O/smoke.log ;;
  bench)
    timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];t=d['timed_runs'];print('bench',round(d['value']),round(d['ms_per_step'],3),t['ms_per_step'],r['kernel'],round(r['frac'],3),'h2d',round(d['h2d']['ms_per_step'],3));print('full',round(d['full_path']['value']),'large',round(d['large']['value']),'cpu',d['cpu_baseline']['value'])" ;;
  distbench)
    VO_BENCH_FORCE_DIST=1 timeout -k 10 600 python3 bench.py --no-cpu --large-batch 0 > $O/distbench.json 2> $O/distbench.err \
      || { tail -20 $O/distbench.err; exit 1; }
    python3 -c "import json;d=json.loads([l for l in open('$O/distbench.json') if l.startswith('{')][0]);f=d['full_path'];print('distbench',d['config']['process_group'],round(d['value']),'full',round(f['value']),f['landmark_rows'],f['accuracy']['ate_rmse_m'])" ;;
  kprof)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kprof -o k -- python3 bench.py --steps 10 --runs 1 --warmup 2 --no-cpu --seq-frames 0 --large-batch 0 > $O/kprof_bench.json 2> $O/kprof.err
    find $O/kprof -name "*kernel_trace.csv" -delete
    echo kprof-done ;;
  seqprof)
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/seqprof -o k -- python3 bench.py --steps 2 --runs 1 --warmup 1 --no-cpu --large-batch 0 > $O/seqprof_bench.json 2> $O/seqprof.err
    find $O/seqprof -name "*kernel_trace.csv" -delete
    echo seqprof-done ;;
  probe:*)
    b=${st#probe:}; timeout -k 10 120 ./tools/$b > $O/$b.txt 2>&1 || { cat $O/$b.txt; exit 1; }
    cat $O/$b.txt ;;
  py:*)
    # py:<tools script>[:args, + for spaces] -- a short python tool on the GPU
    a=${st#py:}; b=${a%%:*}; x=""; [ "$a" != "$b" ] && x=${a#*:}
    timeout -k 10 300 python3 tools/$b ${x//+/ } > $O/${b%.py}.txt 2>&1 || { tail -20 $O/${b%.py}.txt; exit 1; }
    tail -5 $O/${b%.py}.txt ;;
  rehearse2)
    # two ranks on this box's one GPU over gloo (the 8-GPU node runs nccl = RCCL): per-rank loop and tail
    VO_BENCH_BACKEND=gloo VO_BENCH_SAME_GPU=1 timeout -k 10 600 python3 bench.py --gpus 2 --no-cpu --large-batch 0 > $O/rehearse2.json 2> $O/rehearse2.err \
      || { tail -20 $O/rehearse2.err; exit 1; }
    python3 -c "import json;d=json.loads([l for l in open('$O/rehearse2.json') if l.startswith('{')][0]);f=d['full_path'];print('rehearse2',d['n_gpus'],round(f['value']),f['landmark_rows'],f['accuracy']['ate_rmse_m'],f['per_rank_ms'])" ;;
  content_pmc)
    # the same counters for the bench's synthetic pairs and for KITTI-00 street frames (content A/B)
    for w in syn street; do
      a=""; [ $w = street ] && a=street
      timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $O/cp_$w -o p --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES -- python3 tools/prof_run.py 64 2 $a > $O/cp_$w.log 2>&1 \
        || { tail -20 $O/cp_$w.log; exit 1; }
      python3 tools/pmc_sum.py $O/cp_$w > $O/cp_$w.txt
      find $O/cp_$w -name "*.csv" -delete
    done
    grep -h "k_desc\|k_orient\|k_refine\|k_seg_emit" $O/cp_*.txt ;;
  abfull:*)
    # configs[1] and the full path (configs[2]) for the default library and each named variant
    v=${st#abfull:}
    for var in default ${v//,/ } default; do
      if [ $var = default ]; then unset VO_LIBPATH; else export VO_LIBPATH=$GRAFT_REPO_ROOT/tools/variants/$var/libvo.so; fi
      timeout -k 10 300 python3 bench.py --no-cpu --large-batch 0 > $O/abf_$var.json 2>/dev/null || { echo "$var failed"; exit 1; }
      python3 -c "import json;d=json.load(open('$O/abf_$var.json'));f=d['full_path'];k=f['kernel_ms_per_step'];print('$var',round(d['value'],1),round(d['ms_per_step'],3),'full',round(f['value'],1),'refine',d['roofline']['kernel_ms_per_step'].get('k_refine'),k.get('k_refine'),'msac',k.get('k_msac'),k.get('k_msac_gen'))"
    done
    unset VO_LIBPATH ;;
  ab:*)
    v=${st#ab:}; timeout -k 10 900 bash tools/variant_bench.sh ${v//,/ } > $O/ab_${v//,/_}.txt 2>&1 || { cat $O/ab_${v//,/_}.txt; exit 1; }
    cat $O/ab_${v//,/_}.txt ;;
  pmc|pmc:*)
    # pmc:<name> also installs the per-launch traffic as profiles/<name> in this box's copy, so a
    # later bench step of the same call reads it (commit the merged gpurun_out copy afterwards)
    timeout -k 10 900 bash tools/pmc_passes.sh _$(basename $O) > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
    python3 tools/pmc_traffic.py gpurun_out/pmc_$(basename $O) $O/pmc_traffic.json > /dev/null
    [ "$st" != pmc ] && cp $O/pmc_traffic.json profiles/${st#pmc:}
    echo pmc-done ;;
  sbusy)
    # per-stream occupancy of the back-to-back loop (tools/stream_busy.py): which stream is critical
    timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/strace -o t -- python3 tools/prof_run.py ${PMC_BATCH:-256} 6 > $O/strace.log 2>&1 \
      || { tail -20 $O/strace.log; exit 1; }
    python3 tools/stream_busy.py $(find $O/strace -name "*kernel_trace.csv" | head -1) > $O/stream_busy.txt
    find $O/strace -name "*.csv" -delete
    cat $O/stream_busy.txt ;;
  seqbusy:*)
    # seqbusy:<frames>:<batch>:<depth>:<skip> -- per-stream occupancy of the full path's pipelined loop
    a=${st#seqbusy:}; IFS=: read -r n b d k <<< "$a"
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/sq_${b}_${d} -o t -- python3 tools/seq_run.py $n $b $d > $O/sq_${b}_$d.log 2>&1 \
      || { tail -20 $O/sq_${b}_$d.log; exit 1; }
    python3 tools/stream_busy.py $(find $O/sq_${b}_${d} -name "*kernel_trace.csv" | head -1) $k > $O/stream_busy_seq_${b}_$d.txt
    find $O/sq_${b}_${d} -name "*.csv" -delete
    grep pass $O/sq_${b}_$d.log; cat $O/stream_busy_seq_${b}_$d.txt ;;
  fcalib)
    # FETCH_SIZE calibration for the feature kernels' access shapes (tools/fetch_calib.hip)
    timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $O/fcal -o f --pmc FETCH_SIZE -- ./tools/fetch_calib > $O/fetch_calib.txt 2>&1 \
      || { tail -20 $O/fetch_calib.txt; exit 1; }
    python3 tools/fetch_calib_sum.py $(find $O/fcal -name "*counter_collection.csv" | head -1) $O/fetch_calib.txt > $O/fetch_calib_sum.txt
    find $O/fcal -name "*.csv" -delete
    cat $O/fetch_calib_sum.txt ;;
  insitu)
    # kernel trace of the asynchronous loop + the counter passes -> tools/insitu_model.py
    timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/itrace -o t -- python3 tools/prof_run.py ${PMC_BATCH:-256} 6 > $O/itrace.log 2>&1 \
      || { tail -20 $O/itrace.log; exit 1; }
    timeout -k 10 900 bash tools/pmc_passes.sh _$(basename $O) > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
    python3 tools/insitu_model.py gpurun_out/pmc_$(basename $O) $(find $O/itrace -name "*kernel_trace.csv" | head -1) $O/insitu.json
    python3 tools/pmc_traffic.py gpurun_out/pmc_$(basename $O) $O/pmc_traffic.json > /dev/null ;;
  batch:*)
    b=${st#batch:}
    for bb in 64 $b 64; do
      timeout -k 10 300 python3 bench.py --no-cpu --seq-frames 0 --large-batch 0 --batch $bb > $O/batch_$bb.json 2>/dev/null || { echo "batch $bb failed"; exit 1; }
      python3 -c "import json;d=json.load(open('$O/batch_$bb.json'));print('batch',$bb,round(d['value'],1),round(d['ms_per_step'],3))"
    done ;;
  attr)
    timeout -k 10 400 python3 tools/fullpath_attr.py 1024 64 > $O/fullpath_attr.json 2> $O/fullpath_attr.err || { tail -20 $O/fullpath_attr.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/fullpath_attr.json'));print('attr',d['ms_per_batch'])" ;;
  *) echo "unknown step $st"; exit 2 ;;
  esac
done
