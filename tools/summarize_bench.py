"""Print the headline and the sub-figures of a bench.py JSON line (tools/gpu.sh bench)."""
import json
import sys


def main(path):
    lines = [l for l in open(path) if l.startswith("{")]
    if not lines:
        print("no JSON line in", path)
        return
    d = json.loads(lines[-1])
    r, t = d.get("roofline", {}), d.get("roofline_tree", {})
    print("headline %.1f %s  %.2f ms/step  tower frac %.3f (%.3f ms/launch)  tree frac %.3f (%.1f us)" % (
        d["value"], d["unit"], d["ms_per_step"], r.get("frac", 0), r.get("mean_launch_ms", 0), t.get("frac", 0),
        t.get("mean_launch_ms", 0) * 1e3))
    ss = d.get("single_stream_kernels")
    if ss:
        print("single stream: tower %.3f ms frac %.3f | tree %.1f us frac %.3f" % (
            ss["tower"]["mean_launch_ms"], ss["tower"]["frac"], ss["tree"]["mean_launch_ms"] * 1e3, ss["tree"]["frac"]))
    for k, v in d.get("sublines", {}).items():
        if "skipped" in v:
            print("%s: skipped (%s)" % (k, v["skipped"]))
            continue
        print("%s: %.1f moves/s  tower frac %.3f  tree frac %.3f (%.1f us)" % (
            k, v["value"], v.get("roofline", {}).get("frac", 0), v.get("roofline_tree", {}).get("frac", 0),
            v.get("roofline_tree", {}).get("mean_launch_ms", 0) * 1e3))
    w = d.get("worker")
    if w:
        print("worker: %.1f moves/s (%.3f of engine), %d games, %d slices" % (
            w["value"], w["worker_over_engine"] or 0, w["finished_games"], w["slices"]))
    tr = d.get("trainer")
    if tr:
        print("trainer: %.2f steps/s" % tr["value"])
    lc = d.get("loop_c4")
    if lc:
        print("loop_c4: %.1f moves/s + %.2f steps/s, %d games, %d slices, push %.1f ms" % (
            lc["moves_per_s"], lc["trainer_steps_per_s"], lc["finished_games"], lc["slices_added"], lc["weight_push_ms"]))
    cb = d.get("cpu_baseline")
    if cb:
        print("cpu_baseline: %.3f moves/s on %d cores" % (cb["value"], cb["cores"]))


if __name__ == "__main__":
    main(sys.argv[1])
