"""Mean of the per-repetition medians of tools/ab_repeat.sh output, per mode and library."""
import collections, re, sys
acc = collections.defaultdict(list)
mode = None
for ln in open(sys.argv[1]):
    m = re.match(r"== rep \d+ (\w+)", ln)
    if m:
        mode = m.group(1); continue
    m = re.match(r"(\S+\.so)\s+median ([\d.]+) ms", ln)
    if m and mode:
        acc[(mode, m.group(1))].append(float(m.group(2)))
base = {}
for (mode, lib), v in sorted(acc.items()):
    mean = sum(v) / len(v)
    base.setdefault(mode, mean)
    print("%-7s %-16s %.4f ms  (%+.2f %% vs first)  n=%d" % (mode, lib, mean, 100 * (mean / base[mode] - 1), len(v)))
