"""Extract the C3-HLAC bin map from the reference's unrolled source (run in the build
container only; the output JSON is committed as a golden fixture).

Parses the ColorCHLAC{,_RI}Estimation::addColorCHLAC_{0,0_bin,1,1_bin} bodies of
color_chlac/include/color_chlac/color_chlac.hpp (the open twin of the binary-only
c3_hlac_core kernel) and records, for every histogram write, which
(neighbour offset k, centre channel c, neighbour channel n) it accumulates.  Channel
order is r, r_, g, g_, b, b_ = 0..5 (Appendix A of SURVEY.md).

Output (tests/golden/binmap_981.json, binmap_117.json): lists of [k, c, n, bin] /
[c, bin] / [c, n, bin] -- data only, no reference text.

Usage: python oracle/gen_binmap.py /root/reference tests/golden
"""
import json
import re
import sys
from pathlib import Path

CH = {"r": 0, "r_": 1, "g": 2, "g_": 3, "b": 4, "b_": 5}
BIN_COND = {"center_bin_r": (0, 1), "center_bin_g": (2, 3), "center_bin_b": (4, 5)}


def function_body(src, cls, name):
    m = re.search(r"pcl::%s<PointT, PointOutT>::%s\s*\(" % (cls, name), src)
    if not m:
        raise SystemExit("function %s::%s not found" % (cls, name))
    i = src.index("{", m.end())
    depth, j = 0, i
    while True:
        if src[j] == "{":
            depth += 1
        elif src[j] == "}":
            depth -= 1
            if depth == 0:
                return src[i + 1:j]
        j += 1


TOK = re.compile(r"DIM_COLOR_1_3|[A-Za-z_][A-Za-z_0-9]*|\d+|\+\+|\+=|[(){}\[\];:.*+=<>!]|->|\S")


def tokens(body):
    body = re.sub(r"//[^\n]*", "", body)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    return TOK.findall(body)


class Parser:
    """Tiny recursive-descent walker over the unrolled add functions."""

    def __init__(self, toks):
        self.t, self.i = toks, 0
        self.writes = []  # (case_k, frozenset of active centre channels, bin, rhs tokens)

    def peek(self, o=0):
        return self.t[self.i + o] if self.i + o < len(self.t) else None

    def take(self, v=None):
        tok = self.t[self.i]
        if v is not None and tok != v:
            raise SyntaxError("expected %r got %r at %d" % (v, tok, self.i))
        self.i += 1
        return tok

    def block(self, case, conds):
        while self.peek() is not None and self.peek() != "}":
            case = self.stmt(case, conds)
        return case

    def stmt(self, case, conds):
        tok = self.peek()
        if tok == "{":
            self.take("{")
            case = self.block(case, conds)
            self.take("}")
            return case
        if tok == "if":
            self.take("if")
            self.take("(")
            var = self.take()
            self.take(")")
            on, off = BIN_COND[var]
            self.stmt(case, conds | {on})
            if self.peek() == "else":
                self.take("else")
                self.stmt(case, conds | {off})
            return case
        if tok == "switch":
            self.take("switch")
            while self.take() != ")":
                pass
            self.take("{")
            c = None
            while self.peek() != "}":
                c = self.stmt(c, conds)
            self.take("}")
            return case
        if tok == "case":
            self.take("case")
            k = int(self.take())
            self.take(":")
            return k
        if tok == "default":
            self.take("default")
            self.take(":")
            return None
        if tok == "break":
            self.take("break")
            self.take(";")
            return case
        if tok == "const":  # local declarations: const int r_ = 1 - r;
            while self.take() != ";":
                pass
            return case
        # output.points[idx].histogram[ <expr> ] (++ | += rhs) ;
        stmt = []
        while self.peek() != ";":
            stmt.append(self.take())
        self.take(";")
        s = " ".join(stmt)
        m = re.match(r"output \. points \[ idx \] \. histogram \[ (DIM_COLOR_1_3 \+ )?(\d+) \] (\+\+|\+=)(.*)$", s)
        if not m:
            raise SyntaxError("unrecognised statement: " + s)
        b = int(m.group(2)) + (495 if m.group(1) else 0)
        self.writes.append((case, frozenset(conds), b, m.group(3), m.group(4).split()))
        return case


def parse(src, cls, name):
    p = Parser(tokens(function_body(src, cls, name)))
    p.block(None, frozenset())
    return p.writes


def nonbin_operands(rhs):
    # rhs like: center_r * r   |  center_r  |  center_r_ * center_g
    s = "".join(rhs)
    m = re.match(r"^center_(r_|g_|b_|r|g|b)(?:\*(center_)?(r_|g_|b_|r|g|b))?$", s)
    if not m:
        raise SyntaxError("rhs " + s)
    c = CH[m.group(1)]
    n = CH[m.group(3)] if m.group(3) else None
    return c, n, bool(m.group(2))


def build(src, cls, zero_bin_fn, dim):
    out = {"zero": [], "auto": [], "first": [], "bin_zero": [], "bin_pairs": [], "bin_first": []}
    for case, conds, b, op, rhs in parse(src, cls, "addColorCHLAC_0"):
        c, n, _ = nonbin_operands(rhs)
        if n is None:
            out["zero"].append([c, b])
        else:
            out["auto"].append([c, n, b])
    for case, conds, b, op, rhs in parse(src, cls, zero_bin_fn):
        cs = sorted(conds)
        if len(cs) == 1:
            out["bin_zero"].append([cs[0], b])
        else:
            out["bin_pairs"].append([cs[0], cs[1], b])
    for case, conds, b, op, rhs in parse(src, cls, "addColorCHLAC_1"):
        c, n, _ = nonbin_operands(rhs)
        out["first"].append([case if dim == 981 else -1, c, n, b])
    for case, conds, b, op, rhs in parse(src, cls, "addColorCHLAC_1_bin"):
        (c,) = tuple(conds)
        n = CH["".join(rhs)]
        out["bin_first"].append([case if dim == 981 else -1, c, n, b])
    for key in out:
        out[key].sort()
    return out


def main():
    ref = Path(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
    dst = Path(sys.argv[2] if len(sys.argv) > 2 else Path(__file__).resolve().parents[1] / "tests" / "golden")
    src = (ref / "color_chlac/include/color_chlac/color_chlac.hpp").read_text()
    maps = {
        981: build(src, "ColorCHLACEstimation", "addColorCHLAC_0_bin", 981),
        117: build(src, "ColorCHLAC_RI_Estimation", "addColorCHLAC_0_bin", 117),
    }
    for dim, m in maps.items():
        m["source"] = "color_chlac/include/color_chlac/color_chlac.hpp (C3HLAC%s inherits these add functions)" % (
            "Estimation" if dim == 981 else "_RI_Estimation")
        m["channel_order"] = ["r", "r_", "g", "g_", "b", "b_"]
        (dst / ("binmap_%d.json" % dim)).write_text(json.dumps(m, indent=0, sort_keys=True))
        print(dim, {k: len(v) for k, v in m.items() if isinstance(v, list)})


if __name__ == "__main__":
    main()
