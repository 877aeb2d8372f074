"""Per-thread CPU time of a child command (Linux /proc): which threads of a run burn the host.

    python tools/thread_cpu.py [--warm S] -- python bench.py --steps 40

Samples /proc/<pid>/task/*/stat after --warm seconds and again at exit-minus-one-sample, and
prints CPU seconds per thread (name = comm) over that window, grouped by name."""
import argparse
import collections
import os
import subprocess
import sys
import time


def sample(pid):
    out = {}
    tdir = f"/proc/{pid}/task"
    try:
        tids = os.listdir(tdir)
    except FileNotFoundError:
        return out
    tck = os.sysconf("SC_CLK_TCK")
    for t in tids:
        try:
            st = open(f"{tdir}/{t}/stat").read()
        except OSError:
            continue
        name = st[st.index("(") + 1:st.rindex(")")]
        f = st[st.rindex(")") + 2:].split()
        out[t] = (name, (int(f[11]) + int(f[12])) / tck)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--warm", type=float, default=20.0)
    ap.add_argument("--every", type=float, default=1.0)
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
    p = subprocess.Popen(cmd)
    t0 = time.time()
    first = None
    last = {}  # tid -> latest sample (threads that exit keep their last value)
    tf = tl = None
    while p.poll() is None:
        time.sleep(a.every)
        s = sample(p.pid)
        if not s:
            continue
        if time.time() - t0 >= a.warm and first is None:
            first, tf = s, time.time()
        elif first is not None:
            last.update(s)
            tl = time.time()
    rc = p.wait()
    if first is None or not last:
        print("window too short", file=sys.stderr)
        sys.exit(rc)
    by = collections.defaultdict(float)
    cnt = collections.Counter()
    for t, (name, cpu) in last.items():
        c0 = first.get(t, (name, 0.0))[1]
        by[name] += cpu - c0
        cnt[name] += 1
    wall = tl - tf
    print(f"window {wall:.1f} s wall, total CPU {sum(by.values()):.1f} s ({sum(by.values()) / wall:.2f} cores)")
    for name, cpu in sorted(by.items(), key=lambda t: -t[1])[:25]:
        print(f"  {name:<20} threads={cnt[name]:<3} cpu={cpu:7.2f} s  ({cpu / wall:.2f} cores)")
    print("top threads:")
    per = []
    for t, (name, cpu) in last.items():
        per.append((cpu - first.get(t, (name, 0.0))[1], t, name))
    for cpu, t, name in sorted(per, reverse=True)[:16]:
        tag = " (main)" if int(t) == p.pid else ""
        print(f"  tid {t:<8} {name:<16}{tag:<8} cpu={cpu:7.2f} s  ({cpu / wall:.2f} cores)")
    sys.exit(rc)


if __name__ == "__main__":
    main()
