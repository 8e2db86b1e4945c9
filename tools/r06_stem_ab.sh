# trainer.DYN_STEM_HIP (dynamics stem on the HIP conv + action stamp) vs MIOpen's 144-channel conv, alternated
O=gpurun_out/r06_stem
mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 300 python tools/bench_trainer.py --per --steps 40 --warmup 6 > $O/off_$r.json 2> $O/off_$r.err || exit 1
  timeout -k 10 300 python tools/bench_trainer.py --per --steps 40 --warmup 6 --hip-stem > $O/on_$r.json 2> $O/on_$r.err || exit 1
  python3 -c "import json;a=json.load(open('$O/off_$r.json'));b=json.load(open('$O/on_$r.json'));print('round $r: miopen stem %.2f  hip stem %.2f steps/s'%(a['value'],b['value']))"
done
