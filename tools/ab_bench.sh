set -o pipefail
for r in ${REPS:-1 2}; do for v in ${VARS:-va vb}; do
FSEM_LIB=$PWD/fast_speech_enhancement_metrics_amd/lib/var/$v.so timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/ab_$v$r.json || exit 1
echo $v $r $(python -c "import json;d=json.load(open('gpurun_out/ab_$v$r.json'));print(d['ms_per_step'], d['roofline']['ms_per_launch'])")
done; done
