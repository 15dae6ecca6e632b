"""Host CPU topology for the CPU-baseline legs of the benchmarks.

BASELINE.md / SURVEY.md §8(d) ask for the reference CPU path on N = the
host's physical cores, with N stated.  This module finds one logical CPU per
physical core (unique (package, core_id) pairs from
/sys/devices/system/cpu/cpu*/topology), restricted to the CPUs this process
may run on (sched_getaffinity), and reads the cgroup CPU quota (cpu.max) so a
report can say when the process was allowed fewer cores than the machine has.
"""
import glob
import os


def _read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def physical_cores(cpus=None):
    """-> list of logical CPU ids, one per physical core (lowest id of each
    core), over `cpus` (default: this process's affinity mask)."""
    if cpus is None:
        cpus = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))
    seen, out = set(), []
    for c in sorted(cpus):
        base = "/sys/devices/system/cpu/cpu%d/topology/" % c
        pkg, core = _read(base + "physical_package_id"), _read(base + "core_id")
        key = (pkg, core) if pkg is not None and core is not None else ("cpu", c)
        if key not in seen:
            seen.add(key)
            out.append(c)
    return out


def machine_physical_cores():
    """Physical cores of the whole machine (all online CPUs, not only ours)."""
    cpus = []
    for p in glob.glob("/sys/devices/system/cpu/cpu[0-9]*"):
        try:
            cpus.append(int(os.path.basename(p)[3:]))
        except ValueError:
            pass
    return len(physical_cores(cpus)) if cpus else (os.cpu_count() or 1)


def cgroup_cpu_quota():
    """CPUs granted by the cgroup v2 / v1 quota, or None when unlimited."""
    v = _read("/sys/fs/cgroup/cpu.max")
    if v:
        q, p = v.split()[:2]
        if q != "max":
            return float(q) / float(p)
        return None
    q, p = _read("/sys/fs/cgroup/cpu/cpu.cfs_quota_us"), _read("/sys/fs/cgroup/cpu/cpu.cfs_period_us")
    if q and p and int(q) > 0:
        return float(q) / float(p)
    return None


def baseline_cpus():
    """-> (cpu ids to pin one worker thread each, description dict).

    One thread per physical core we may run on; if a cgroup quota grants
    fewer CPUs than that, only as many threads as the quota (more threads
    would time-slice and understate the per-core rate)."""
    phys = physical_cores()
    quota = cgroup_cpu_quota()
    use = phys
    if quota is not None and int(quota) < len(phys):
        use = phys[:max(1, int(quota))]
    info = {"machine_physical_cores": machine_physical_cores(), "allowed_physical_cores": len(phys),
            "cgroup_cpu_quota": quota, "threads": len(use), "pinned": True}
    return use, info
