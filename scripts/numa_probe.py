"""Prints what the box shows about CPU / GPU NUMA placement (no GPU call):
the visible-device variables, each AMD render node's NUMA node and whether
this process may open it, each NUMA node's CPU list, and this process's
allowed CPUs."""
import glob
import os

for k, v in sorted(os.environ.items()):
    if "VISIBLE" in k or k in ("OMP_NUM_THREADS",):
        print("env", k, v)
for r in sorted(glob.glob("/sys/class/drm/renderD*")):
    dev = os.path.basename(r)
    try:
        numa = open(os.path.join(r, "device", "numa_node")).read().strip()
        vendor = open(os.path.join(r, "device", "vendor")).read().strip()
    except OSError:
        continue
    print("render", dev, "vendor", vendor, "numa", numa, "open", os.access("/dev/dri/" + dev, os.R_OK | os.W_OK))
for n in sorted(glob.glob("/sys/devices/system/node/node*")):
    print("node", os.path.basename(n), open(os.path.join(n, "cpulist")).read().strip())
print("allowed", len(os.sched_getaffinity(0)))
for line in open("/proc/self/status"):
    if line.startswith("Cpus_allowed_list") or line.startswith("Mems_allowed_list"):
        print(line.strip())
for p in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpuset.cpus.effective"):
    try:
        print(p, open(p).read().strip())
    except OSError:
        pass
