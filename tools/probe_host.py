"""Dev probe: the GPU box's host CPU resources as a process sees them (bench.py cpu_baseline)."""
import os

print("os.cpu_count", os.cpu_count())
print("sched_getaffinity", len(os.sched_getaffinity(0)))
for p in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us",
          "/sys/fs/cgroup/cpu/cpu.cfs_period_us", "/sys/fs/cgroup/cpuset.cpus.effective"):
    try:
        print(p, open(p).read().strip())
    except OSError as e:
        print(p, "-", e.__class__.__name__)
for k in ("OMP_NUM_THREADS", "MAX_JOBS"):
    print(k, os.environ.get(k))
try:
    for line in open("/proc/cpuinfo"):
        if line.startswith("model name"):
            print(line.strip())
            break
except OSError:
    pass
