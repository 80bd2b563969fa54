# GPU-box helper: A/B of the in-tree library against variant builds var_<name>.so (repo root),
# configs[2] and configs[4] bench lines twice each.  usage: tools/ab_variant.sh <name>...
set -o pipefail
mkdir -p gpurun_out
for v in default "$@" default "$@"; do
  if [ $v = default ]; then L=$PWD/your-voice-tts_amd/libtts_hip.so; else L=$PWD/var_$v.so; fi
  TTS_HIP_LIB=$L timeout -k 10 200 python bench.py --batch 64 --lengths uniform --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail -20 gpurun_out/ab_$v.err; exit 1; }
  TTS_HIP_LIB=$L timeout -k 10 200 python bench.py --model gst --batch 32 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/abg_$v.json 2> gpurun_out/abg_$v.err || { tail -20 gpurun_out/abg_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));s=d['stages_rank0'];e=[json.loads(l) for l in open('gpurun_out/abg_$v.json') if l.startswith('{')][0];print('$v',round(d['value']),round(s['tacotron2_ms']-s['decoder_loop_ms'],2),round(e['value']),round(e['stages_rank0']['tacotron2_ms']-e['stages_rank0']['decoder_loop_ms'],2))"
done
