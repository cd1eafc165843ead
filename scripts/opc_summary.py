"""Summary of scripts/gpu_opcost.sh: per form, the SQ instruction mix per
wave-step of the measured (second) run, whose k_run is the last dispatch of
the case's group in the counter CSV, next to op_cost.py's timing."""
import collections
import csv
import json
import sys

KEYS = ["SQ_INSTS_SALU", "SQ_INSTS_VALU", "SQ_INSTS_BRANCH", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
        "SQ_INSTS_SMEM"]


def main(d):
    rows = list(csv.reader(open(f"{d}/k_run_counters.csv")))
    disp = collections.OrderedDict()
    for r in rows:
        disp.setdefault(int(r[1]), {})[r[15]] = float(r[16])
    ids = sorted(disp)
    cases = [json.loads(x) for x in open(f"{d}/times.jsonl")]
    # each case: the first run's regrouped launches end with near-empty ones
    # (the lanes already stopped), then the measured run's single launch
    small = [disp[i].get("SQ_INSTS_SALU", 0) < 1e6 for i in ids]
    measured = [ids[k] for k in range(1, len(ids)) if small[k - 1] and not small[k]]
    assert len(measured) == len(cases), (len(measured), len(cases))
    out = []
    for c, did in zip(cases, measured):
        m = disp[did]
        ws = c["wave_steps"]
        per = {k: m.get(k, 0) / ws for k in KEYS}
        out.append((c["case"], sum(per.values()), per, c["ns_per_wave_step"]))
    print("case        instr  salu  valu   br  lds  vmrd vmwr ns/ws cyc/instr")
    for name, tot, p, ns in out:
        print(f"{name:10s} {tot:6.0f} {p['SQ_INSTS_SALU']:5.0f} {p['SQ_INSTS_VALU']:5.0f} {p['SQ_INSTS_BRANCH']:4.0f} "
              f"{p['SQ_INSTS_LDS']:4.1f} {p['SQ_INSTS_VMEM_RD']:4.2f} {p['SQ_INSTS_VMEM_WR']:4.2f} {ns:5.0f} "
              f"{ns * 2.4 / max(tot, 1):5.1f}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/opc")
