#!/usr/bin/env python3
"""VALU instructions per loop iteration of every kernel in tools/microbench_mac.hip, read from the gfx950
assembly (hipcc --save-temps): the microbench's 'other VALU' rates use these counts, not nominal ones."""
import collections
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    with tempfile.TemporaryDirectory() as d:
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-c", "--save-temps", "-o",
                               os.path.join(d, "m.o"), os.path.join(ROOT, "tools", "microbench_mac.hip")], cwd=d,
                              stderr=subprocess.DEVNULL)
        s = open(glob.glob(os.path.join(d, "*gfx950.s"))[0]).read()
    out = {}
    for m in re.finditer(r"^(_Z\w+):", s, re.M):
        name = m.group(1)
        body = s[m.end():s.find("s_endpgm", m.end())]
        lm = re.search(r"^(\.LBB\w+):.*?$(.*?)s_cbranch_scc1 \1", body, re.M | re.S)
        if not lm:
            continue
        loop = lm.group(2)
        step = re.search(r"s_add_i32 s\d+, s\d+, -(\d+)", loop)
        unroll = int(step.group(1)) if step else 1
        ops = collections.Counter(x.group(1) for x in re.finditer(r"^\s*(v_\w+)", loop, re.M))
        mac = ops.pop("v_mad_u64_u32", 0)
        other = sum(ops.values())
        dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        out[dem] = (mac / unroll, other / unroll, unroll)
        print("%-40s unroll %d  MAC/iter %.2f  other VALU/iter %.2f  %s" % (dem, unroll, mac / unroll, other / unroll,
                                                                         dict(ops)))
    return out


if __name__ == "__main__":
    main()
