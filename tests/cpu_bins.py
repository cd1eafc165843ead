"""Where the CPU-side test binaries live. In-tree by default (oracle/,
tests/native/); WTF_CPU_BUILD=<dir> selects another build of the same sources
instead (scripts/sanitize_cpu.sh: AddressSanitizer + UndefinedBehaviorSanitizer),
which is then used as it is: nothing is rebuilt in-tree."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ALT = os.environ.get("WTF_CPU_BUILD") or None


def _path(default: str) -> str:
    return os.path.join(ALT, os.path.basename(default)) if ALT else default


ORACLE_SO = _path(os.path.join(ROOT, "oracle", "liboracle.so"))
TWIN = _path(os.path.join(ROOT, "oracle", "wtf_twin"))
HOSTCHECK = _path(os.path.join(ROOT, "oracle", "hostcheck"))
SIMLANE_SO = _path(os.path.join(ROOT, "tests", "native", "libsimlane.so"))


def ensure(path: str, make_dir: str, target: str | None = None) -> str:
    """The in-tree binary is (re)made by its Makefile; an alternative build is taken as it is."""
    if not ALT:
        subprocess.check_call(["make", "-s", "-C", make_dir] + ([target] if target else []))
    return path
