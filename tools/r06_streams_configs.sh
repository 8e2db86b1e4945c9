# one vs two streams (tower cap all-but-32 vs 3/4) for C1 (9x9 AlphaZero/50) and C5 (19x19/800/16 blocks), alternated
O=gpurun_out/r06_streams
mkdir -p $O
for r in 1 2; do
  for v in "1 0" "2 224" "2 192"; do
    set -- $v
    timeout -k 10 300 python3 tools/dual_stream_probe.py --size 9 --sims 50 --mode AlphaZero --parts $1 --max-grid $2 --moves 20 --warmup 3 > $O/c1_$1_$2_$r.json 2> $O/c1_$1_$2_$r.err || { echo "c1 $v failed"; tail -3 $O/c1_$1_$2_$r.err; exit 1; }
    echo "C1 parts $1 cap $2: $(python3 -c "import json;print('%.0f'%json.load(open('$O/c1_$1_$2_$r.json'))['moves_per_s'])") moves/s"
  done
done
for r in 1 2; do
  for v in "1 0" "2 224"; do
    set -- $v
    timeout -k 10 400 python3 tools/dual_stream_probe.py --size 19 --sims 800 --blocks 16 --parts $1 --max-grid $2 --moves 2 --warmup 1 > $O/c5_$1_$2_$r.json 2> $O/c5_$1_$2_$r.err || { echo "c5 $v failed"; tail -3 $O/c5_$1_$2_$r.err; exit 1; }
    echo "C5 parts $1 cap $2: $(python3 -c "import json;print('%.0f'%json.load(open('$O/c5_$1_$2_$r.json'))['moves_per_s'])") moves/s"
  done
done
