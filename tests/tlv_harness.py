"""Drives `wtfgpu` (the product node, wtf_amd/host) and `oracle/wtf_twin`
(its CPU twin) over the synthetic tlv_server and HEVD snapshots."""
from __future__ import annotations

import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WTFGPU = os.path.join(ROOT, "wtf_amd", "host", "wtfgpu")
from tests.cpu_bins import TWIN  # noqa: E402


def build_hevd_target(d: str) -> str:
    from wtf_amd.tools.hevd import build, seed_inputs
    build(os.path.join(d, "state"), os.path.join(d, "work"))
    seed_inputs(os.path.join(d, "inputs"))
    return d


def build_hevd_io_target(d: str) -> str:
    """The hevd leg's snapshot: the I/O manager's IRP path (wtf_amd/tools/hevd_io.py)."""
    from wtf_amd.tools.hevd_io import build, seed_inputs
    build(os.path.join(d, "state"), os.path.join(d, "work"))
    seed_inputs(os.path.join(d, "inputs"))
    return d


def build_target(d: str) -> str:
    from wtf_amd.tools.tlv import build, seed_inputs
    build(os.path.join(d, "state"), os.path.join(d, "work"))
    seed_inputs(os.path.join(d, "inputs"))
    return d


def run(exe: str, target: str, inputs: str, results: str, lanes: int, limit: int = 100000,
        full_coverage: bool = True, timeout: int = 300, extra=(), name: str = "tlv_server",
        env: dict | None = None) -> list[dict]:
    cmd = [exe, "run", "--name", name, "--target", target, "--input", inputs, "--results", results,
           "--lanes", str(lanes), "--limit", str(limit), *extra]
    if full_coverage:
        cmd.append("--full-coverage")
    subprocess.run(cmd, check=True, timeout=timeout, env=None if env is None else {**os.environ, **env})
    with open(results) as f:
        return [json.loads(line) for line in f]


def fuzz(exe: str, target: str, runs: int, lanes: int, seed: int = 1337, limit: int = 100000,
         seconds: float = 0, timeout: int = 600, name: str = "tlv_server", max_len: int = 0x1000,
         extra=()) -> dict:
    cmd = [exe, "fuzz", "--name", name, "--target", target, "--runs", str(runs), "--lanes", str(lanes),
           "--seed", str(seed), "--limit", str(limit), "--max_len", str(max_len), *extra]
    if seconds:
        cmd += ["--seconds", str(seconds)]
    out = subprocess.run(cmd, check=True, timeout=timeout, capture_output=True, text=True).stdout
    return json.loads([line for line in out.splitlines() if line.startswith("{")][-1])
