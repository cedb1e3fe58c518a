#!/bin/bash
# GPU box: the alignment GPU tests on the FFT fine-search variant (lib/var/ffine.so) and the three
# aligned-PESQ bench workloads on the direct (dfine) and FFT (ffine) variants.
set -o pipefail
mkdir -p gpurun_out/ff
V=$PWD/fast_speech_enhancement_metrics_amd/lib/var
FSEM_LIB=$V/ffine.so timeout -k 10 400 python -u -m pytest tests/test_align_gpu.py tests/test_align_utt_gpu.py tests/test_align_p862_gpu.py tests/test_bad_intervals_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/ff/tests.log 2>&1
echo "tests rc=$?"
tail -15 gpurun_out/ff/tests.log
for lib in dfine ffine; do for w in pesq_aligned pesq_aligned_utt pesq_aligned_p862; do
  FSEM_LIB=$V/$lib.so timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/ff/${lib}_$w.json 2> gpurun_out/ff/${lib}_$w.err || { echo "bench $lib $w failed"; tail -5 gpurun_out/ff/${lib}_$w.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ff/${lib}_$w.json'));print('$lib $w', d['ms_per_step'], d.get('delays_recovered'))"
done; done
