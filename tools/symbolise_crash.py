"""Attribute the native frames of round 3's rocprofv3 farm crash
(profiles/r3/farm_rocprof_crash.txt) to shared objects, from a map of the
same command's process captured in round 4 (tools/farm_prof.py --maps,
gpurun_out/r4h/maps_w8ng.json).

Linux randomises the mmap base once per process; objects mapped in the same
order keep their distances.  The crash stack holds the signal trampoline
`__restore_rt` (glibc 2.35: libc + 0x42520), which anchors libc's base in
the crashed process; every other frame is placed by its distance from libc
in the captured map and named by the nearest exported symbol of that object
in this image (the same ROCm 7.2 / torch build as the GPU box).

    python tools/symbolise_crash.py MAPS.json > profiles/r4/farm_rocprof_crash_symbolised.txt
"""
import bisect
import json
import subprocess
import sys

FRAMES = [  # profiles/r3/farm_rocprof_crash.txt, innermost first (PC, then the stack)
    ("PC", 0x75a6cb6392fb),
    ("#0", 0x75a6cb185ee8), ("#1", 0x75a6cc04a50e), ("#2", 0x75a6cb12e520), ("#3", 0x75a6cb6392fb),
    ("#4", 0x75a6c0b50266), ("#5", 0x75a6c0b415c0), ("#6", 0x75a5f62cac1a), ("#7", 0x75a5f62c6f89),
    ("#8", 0x75a5f62c7615), ("#9", 0x75a5f6291635), ("#10", 0x75a5f6150475), ("#11", 0x75a5f619c284),
    ("#12", 0x75a5f61509ea), ("#13", 0x75a5f61679b1), ("#14", 0x75a6cb999ec0),
    ("#15", 0x75a547fbfb3f),  # Trlan<false>::orth (libedgpu.so, symbolised in the crash log)
]
RESTORE_RT = 0x75a6cb12e520
RESTORE_RT_OFF = 0x42520  # glibc 2.35 __restore_rt


def dyn_symbols(path, cache={}):
    if path not in cache:
        out = subprocess.run(["nm", "-D", "--defined-only", "-C", path], capture_output=True, text=True).stdout
        s = []
        for ln in out.splitlines():
            f = ln.split(" ", 2)
            if len(f) == 3 and f[1] in "TtWw":
                s.append((int(f[0], 16), f[2]))
        cache[path] = sorted(s)
    return cache[path]


def main():
    maps = json.load(open(sys.argv[1]))
    libc = int(maps["/usr/lib/x86_64-linux-gnu/libc.so.6"]["base"], 16)
    spans = []
    for path, v in maps.items():
        base = int(v["base"], 16)
        for lo, hi, _ in v["exec"]:
            spans.append((int(lo, 16) - libc, int(hi, 16) - libc, base - libc, path))
    libc_r3 = RESTORE_RT - RESTORE_RT_OFF
    print("# round-3 crash frames placed by their distance from libc (anchor: __restore_rt = libc+0x42520)")
    print("# frame  address  object  offset  nearest exported symbol (internal functions: large offsets)")
    for tag, a in FRAMES:
        rel = a - libc_r3
        hit = [(p, rel - b) for lo, hi, b, p in spans if lo <= rel < hi]
        if not hit:
            print(f"{tag:4s} {a:#x}  (not in an object of the captured map: libedgpu.so was rebuilt since)")
            continue
        path, off = hit[0]
        syms = dyn_symbols(path)
        i = bisect.bisect_right([x for x, _ in syms], off) - 1
        near = f"{syms[i][1][:80]} + {off - syms[i][0]:#x}" if i >= 0 else "?"
        print(f"{tag:4s} {a:#x}  {path}  {off:#x}  {near}")


if __name__ == "__main__":
    main()
