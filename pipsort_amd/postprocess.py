"""Post-processing of PIPSORT outputs: global and
not-shared PIPs, the last two steps of the reference's example pipeline
(tests/example/run_example.sh:3-5).

    python -m pipsort_amd.postprocess global  <study0_post> <study1_post> <shared_pips> <out>
    python -m pipsort_amd.postprocess notshared <shared_pips> <global_pips> <out>

Same inputs, outputs and checks as utils/get_global_pips.py and
utils/get_not_shared_pips.py, without pandas:

* global_pips = PIP_study0 + PIP_study1 - shared_pip per union SNP
  (get_global_pips.py:23; a SNP absent from a study contributes 0, :21-22),
  rows in the lexicographic SNP order of the two-study outer join (:18),
  columns SNP_ID, shared_ll, notshared_ll, global_pips (:35);
* not_shared_pip = global_pips - shared_pip (get_not_shared_pips.py:30), rows
  in the global file's order, the LL columns of both files kept with pandas'
  _x / _y suffixes (:29, :35);
* tab-separated, numbers written the way pandas writes them (shortest
  round-trip repr for floats, integers for all-integer columns);
* the reference's range assertions (global in [0, 1] within 1e-6,
  get_global_pips.py:32-33; not-shared / shared, get_not_shared_pips.py:31-34)
  raise ValueError.

These are O(N) host passes over a few hundred lines; there is no device work.
"""
from __future__ import annotations

import math
import sys

__all__ = ["global_pips", "not_shared_pips", "main"]


class _Col:
    """A parsed column: values plus pandas' dtype inference (int64 when every
    cell is an integer literal and nothing is missing, else float64)."""

    def __init__(self, vals, is_int):
        self.vals = vals
        self.is_int = is_int


_E10 = [float(f"1e{k}") for k in range(309)]  # correctly rounded 10^k, as C literals


def _pd_strtod(tok: str) -> float:
    """The float parser pandas' read_csv uses by default (C engine,
    float_precision=None -> precise_xstrtod in pandas/_libs/src/parser/
    tokenizer.c, pandas 2.x; the reference utils run on pandas 2.3.3, SURVEY
    §8(c)): up to 17 significant digits accumulated in a double, then ONE
    multiply or divide by a table power of ten.  Not always correctly rounded,
    so Python's float() would differ from the reference by an ulp."""
    p, n = 0, len(tok)
    while p < n and tok[p] == " ":
        p += 1
    neg = False
    if p < n and tok[p] in "+-":
        neg = tok[p] == "-"
        p += 1
    number, exponent, digits, decimals = 0.0, 0, 0, 0
    while p < n and tok[p].isdigit():
        if digits < 17:
            number = number * 10.0 + (ord(tok[p]) - 48)
            digits += 1
        else:
            exponent += 1
        p += 1
    if p < n and tok[p] == ".":
        p += 1
        while digits < 17 and p < n and tok[p].isdigit():
            number = number * 10.0 + (ord(tok[p]) - 48)
            p += 1
            digits += 1
            decimals += 1
        while p < n and tok[p].isdigit():
            p += 1
        exponent -= decimals
    if digits == 0:
        raise ValueError(f"not a number: {tok!r}")
    if neg:
        number = -number
    if p < n and tok[p] in "eE":
        p += 1
        eneg = False
        if p < n and tok[p] in "+-":
            eneg = tok[p] == "-"
            p += 1
        e = 0
        while p < n and tok[p].isdigit():
            e = e * 10 + (ord(tok[p]) - 48)
            p += 1
        exponent += -e if eneg else e
    if exponent > 308:
        return math.copysign(math.inf, number)
    if exponent > 0:
        return number * _E10[exponent]
    if exponent < -308:
        if exponent < -616:
            return 0.0 * number
        return number / _E10[-308 - exponent] / _E10[308]
    return number / _E10[-exponent]


def _parse_num(tok: str):
    t = tok.strip()
    if t.lstrip("+-").isdigit():
        return int(t), True
    return _pd_strtod(t), False


def _read(path):
    with open(path) as f:
        lines = [l.rstrip("\n").rstrip("\r") for l in f if l.strip()]
    head = lines[0].split("\t")
    rows = [l.split("\t") for l in lines[1:]]
    keys = [r[0] for r in rows]
    cols = {}
    for j, name in enumerate(head[1:], start=1):
        parsed = [_parse_num(r[j]) for r in rows]
        is_int = all(p[1] for p in parsed)
        cols[name] = _Col([float(p[0]) if not is_int else p[0] for p in parsed], is_int)
    return head[0], keys, cols


def _fmt(v, is_int):
    if is_int:
        return str(int(v))
    return repr(float(v))


def _close(a, b, atol):
    # numpy.isclose(a, b, atol=atol) with the default rtol = 1e-5
    return abs(a - b) <= atol + 1e-5 * abs(b)


def global_pips(study0_post: str, study1_post: str, shared_pips: str, out: str):
    """utils/get_global_pips.py: study posts + shared PIPs -> global PIPs file."""
    _, k0, c0 = _read(study0_post)
    _, k1, c1 = _read(study1_post)
    _, ks, cs = _read(shared_pips)
    p0 = dict(zip(k0, c0["Prob_in_pCausalSet"].vals))
    p1 = dict(zip(k1, c1["Prob_in_pCausalSet"].vals))
    union = sorted(set(k0) | set(k1))  # the outer join sorts its keys (get_global_pips.py:18)
    if len(union) != len(ks):
        raise ValueError("study posts and shared PIPs cover different SNP sets (get_global_pips.py:19)")
    srow = {k: i for i, k in enumerate(ks)}
    missing = len(union) != len(k0) or len(union) != len(k1)
    x_int = c0["Prob_in_pCausalSet"].is_int and not (set(k1) - set(k0))
    y_int = c1["Prob_in_pCausalSet"].is_int and not (set(k0) - set(k1))
    sp, sll, nsll = cs["shared_pip"], cs["shared_ll"], cs["notshared_ll"]
    g_int = x_int and y_int and sp.is_int and not missing
    lines = ["SNP_ID\tshared_ll\tnotshared_ll\tglobal_pips"]
    for k in union:
        if k not in srow:  # inner join with the shared file drops it (get_global_pips.py:20)
            continue
        i = srow[k]
        x = p0.get(k, 0)
        y = p1.get(k, 0)
        g = (x + y) - sp.vals[i]
        if not ((g <= 1.0) or _close(g, 1.0, 1e-6)) or not ((g >= 0) or _close(g, 0.0, 1e-6)):
            raise ValueError(f"global PIP of {k} outside [0, 1]: {g} (get_global_pips.py:32-33)")
        lines.append("\t".join([k, _fmt(sll.vals[i], sll.is_int), _fmt(nsll.vals[i], nsll.is_int), _fmt(g, g_int)]))
    with open(out, "w") as f:
        f.write("\n".join(lines) + "\n")


def not_shared_pips(shared_pips: str, global_pips_file: str, out: str):
    """utils/get_not_shared_pips.py: global PIPs - shared PIPs."""
    _, ks, cs = _read(shared_pips)
    _, kg, cg = _read(global_pips_file)
    if len(ks) != len(kg):
        raise ValueError("shared and global PIP files differ in length (get_not_shared_pips.py:28)")
    srow = {k: i for i, k in enumerate(ks)}
    sp = cs["shared_pip"]
    gp = cg["global_pips"]
    n_int = gp.is_int and sp.is_int
    lines = ["SNP_ID\tshared_ll_x\tnotshared_ll_x\tshared_ll_y\tnotshared_ll_y\tnot_shared_pip"]
    for j, k in enumerate(kg):
        if k not in srow:
            continue
        i = srow[k]
        ns = gp.vals[j] - sp.vals[i]
        s = sp.vals[i]
        if not (ns <= 1) or not ((ns >= 0) or _close(ns, 0.0, 1e-6)):
            raise ValueError(f"not-shared PIP of {k} outside [0, 1]: {ns} (get_not_shared_pips.py:31-32)")
        if not (s <= 1) or not ((s >= 0) or _close(s, 0.0, 1e-6)):
            raise ValueError(f"shared PIP of {k} outside [0, 1]: {s} (get_not_shared_pips.py:33-34)")
        lines.append("\t".join([k, _fmt(cg["shared_ll"].vals[j], cg["shared_ll"].is_int),
                                _fmt(cg["notshared_ll"].vals[j], cg["notshared_ll"].is_int),
                                _fmt(cs["shared_ll"].vals[i], cs["shared_ll"].is_int),
                                _fmt(cs["notshared_ll"].vals[i], cs["notshared_ll"].is_int), _fmt(ns, n_int)]))
    with open(out, "w") as f:
        f.write("\n".join(lines) + "\n")


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if argv and argv[0] == "global" and len(argv) == 5:
        global_pips(*argv[1:])
    elif argv and argv[0] == "notshared" and len(argv) == 4:
        not_shared_pips(*argv[1:])
    else:
        print(__doc__.split("\n\n")[1], file=sys.stderr)
        return 2
    return 0


if __name__ == "__main__":
    sys.exit(main())
