"""Extract the rotateFeature90 index maps from the reference's source (run in the build
container only; the output JSON is committed as a golden fixture).

Parses the four `case R_MODE_k:` blocks of pcl::rotateFeature90
(c3_hlac/src/c3_hlac.cpp:49-172) -- assignments of the form
    output[ a + <i or j>*s + <j or i>*78 ] = input[ b + i*s + j*78 ];
inside `for i, for j in 0..5` -- and evaluates them, giving per mode the map
out_index -> in_index over the first-order block 6..473 of one 495- or 486-dim half
(indices 0..5 and 474.. are copied unchanged by the function).

Output (tests/golden/rotate90_map.json): {"R_MODE_1": [474 ints], ...} with
map[o] = the input index written to output o (-1 if none) -- data only, no reference
text.

Usage: python oracle/gen_rotmap.py /root/reference tests/golden
"""
import json
import re
import sys
from pathlib import Path

ASSIGN = re.compile(r"output\[\s*(\d+)\s*\+\s*([ij])\*(\d+)\s*\+\s*([ij])\*78\s*\]\s*=\s*"
                    r"input\[\s*(\d+)\s*\+\s*([ij])\*(\d+)\s*\+\s*([ij])\*78\s*\]")


def extract(src):
    start = src.index("void pcl::rotateFeature90")
    body = src[start:src.index("functions for C3HLACSignature117", start)]
    modes = {}
    parts = re.split(r"case (R_MODE_\d):", body)
    for name, text in zip(parts[1::2], parts[2::2]):
        text = text.split("break;")[0]
        m = [-1] * 474
        n = 0
        for a, u1, s1, u2, b, v1, s2, v2 in ASSIGN.findall(text):
            for i in range(6):
                for j in range(6):
                    env = {"i": i, "j": j}
                    o = int(a) + env[u1] * int(s1) + env[u2] * 78
                    src_i = int(b) + env[v1] * int(s2) + env[v2] * 78
                    if m[o] != -1:
                        raise SystemExit("%s: output %d written twice" % (name, o))
                    m[o] = src_i
            n += 1
        if n != 13:
            raise SystemExit("%s: %d assignments (expected 13)" % (name, n))
        modes[name] = m
    if sorted(modes) != ["R_MODE_1", "R_MODE_2", "R_MODE_3", "R_MODE_4"]:
        raise SystemExit("modes found: %s" % sorted(modes))
    return modes


def main():
    ref, out = Path(sys.argv[1]), Path(sys.argv[2])
    src = (ref / "c3_hlac/src/c3_hlac.cpp").read_text()
    modes = extract(src)
    for name, m in modes.items():
        assert all(v >= 0 for v in m[6:]), name
        assert sorted(m[6:]) == list(range(6, 474)), name  # a permutation of the block
    (out / "rotate90_map.json").write_text(json.dumps(modes, separators=(",", ":")) + "\n")
    print("wrote", out / "rotate90_map.json")


if __name__ == "__main__":
    main()
