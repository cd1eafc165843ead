"""Condensed view of a bench.py JSON line: headline, kernel busy, the step
thread's per-step split (node_timed) and the legs."""
import json
import sys


def per_step(t, steps, keys):
    return " ".join(f"{k}={t.get(k, 0) / steps:.2f}" for k in keys if k in t)


def main(path):
    d = json.loads([x for x in open(path) if x.startswith("{")][-1])
    st = d["steps"]
    print(f"tlv value={d['value'] / 1e6:.3f}M ms/step={d['ms_per_step']:.2f} busy={d.get('kernel_busy_frac', 0):.2f} "
          f"hostcpu={d.get('host_cpu_frac', 0):.2f} frac={d['roofline']['frac']:.4f} "
          f"launch={d['roofline']['avg_launch_ms']:.3f}ms lpws={d['lanes_per_wave_step']:.1f}")
    t = d.get("node_timed", {})
    b = t.get("backend", {})
    print("  node/step:", per_step(t, st, ["step_ms", "fill_ms", "account_ms", "produce_wait_ms", "make_ms", "cpu_s",
                                           "mutate_cpu_ms"]))
    print("  backend/step:", per_step(b, st, ["kernel_ms", "run_ms", "harvest_ms", "exits_ms", "coverage_ms",
                                              "target_restore_ms", "insert_ms", "restore_ms", "restore_dev_ms",
                                              "module_ms", "upload_ms", "up_prep_ms", "up_feed_ms", "fresh_ms",
                                              "occ_ms", "prepared"]))
    for leg in ("hevd", "hevd_bare"):
        h = d.get(leg)
        if not h:
            continue
        hb = h["backend"]
        w = h["wall_s"] * 1e3
        print(f"{leg} value={h['value'] / 1e6:.3f}M busy={h['kernel_busy_frac']:.2f} errors={h['errors']} "
              f"instr/exec={h['instr_per_exec']:.0f} crash={h.get('crash_share', 0):.3f} "
              f"lpws={h['lanes_per_wave_step']:.1f} "
              f"frac={h['roofline']['frac']:.4f} launch={h['roofline']['avg_launch_ms']:.3f}ms "
              f"insert={hb['insert_ms'] / w:.2f} harvest={hb['harvest_ms'] / w:.2f} "
              f"account={h['node']['account_ms'] / w:.2f} (fractions of wall)")
    s = d.get("syn")
    if s:
        print(f"syn value={s['value'] / 1e6:.3f}M ms/step={s['ms_per_step']:.2f} launch={s['roofline']['avg_launch_ms']:.2f}ms "
              f"lpws={s['lanes_per_wave_step']:.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
