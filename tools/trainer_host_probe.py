"""Host-side time of the trainer loop (bench_trainer form: sample, step with the logs read one step late,
priority update) on C4: shows whether the host or the GPU bounds the step (the logs read waits for the GPU)."""
import sys, time, numpy as np, torch
sys.path.insert(0, '.')
from datou_gomoku_muzero_amd import trainer as T
cfg = T.TrainConfig(BOARD_SIZE=15, NUM_RES_BLOCKS=8, PHYSICAL_BATCH_SIZE=360, TRAIN_BUFFER_SIZE=4096, ENABLE_PER=True)
from datou_gomoku_muzero_amd import weights as W
rb = T.ReplayBuffer(cfg, device="cuda"); rs = np.random.RandomState(0)
rb.add_arrays(*W.synthetic_slices(4096, 15, cfg.NUM_UNROLL_STEPS, rs))
tr = T.Trainer(cfg, device="cuda")
pend = None
for i in range(12):
    t0 = time.perf_counter(); batch, idx, w = rb.sample(360, rs); t1 = time.perf_counter()
    logs, td = tr.step(batch, w, sync=False); t2 = time.perf_counter()
    rb.update_priorities(idx, td); t3 = time.perf_counter()
    if pend is not None: pend.tolist()
    t4 = time.perf_counter(); pend = logs
    if i >= 6: print("sample %.2f ms  step %.2f ms  update %.2f ms  logs-read %.2f ms" % ((t1-t0)*1e3, (t2-t1)*1e3, (t3-t2)*1e3, (t4-t3)*1e3))
