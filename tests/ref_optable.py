"""Reads the (op, type) availability pattern straight from the text of the
reference's ompi/mca/op/base/op_base_functions.c (TEST INFRASTRUCTURE).

The kernel tables (ompi_op_base_functions :1485-1569,
ompi_op_base_3buff_functions :1572-1655) are designated initialisers built
from group macros (C_INTEGER, FORTRAN_INTEGER, FLOATING_POINT, LOGICAL,
COMPLEX, BYTE, TWOLOC, :1287-1470) whose entries are NULL unless a configure
switch (OMPI_HAVE_FORTRAN_*, HAVE_SHORT_FLOAT, ...) is set.  This module
expands exactly that: the function-like #defines of the file, the #if/#else
blocks around them under a given configuration, and the table rows -- a
reading of the reference, nothing of it is compiled.  A slot is available
when its initialiser expands to a function name rather than NULL.
"""
import os
import re

SRC = "/root/reference/ompi/mca/op/base/op_base_functions.c"

OPS = ["NULL", "MAX", "MIN", "SUM", "PROD", "LAND", "BAND", "LOR", "BOR", "LXOR", "BXOR", "MAXLOC", "MINLOC",
       "REPLACE", "NO_OP"]


def config(fortran):
    """The configure result of the two table variants:
    C only, or Fortran INTEGER(1,2,4,8) / REAL(4,8) / DOUBLE PRECISION /
    LOGICAL present; never INTEGER16, REAL2, REAL16 or short float."""
    v = 1 if fortran else 0
    c = {f"OMPI_HAVE_FORTRAN_{k}": v for k in ("INTEGER", "INTEGER1", "INTEGER2", "INTEGER4", "INTEGER8", "REAL",
                                                 "REAL4", "REAL8", "DOUBLE_PRECISION", "LOGICAL")}
    c.update({"OMPI_HAVE_FORTRAN_INTEGER16": 0, "OMPI_HAVE_FORTRAN_REAL2": 0, "OMPI_HAVE_FORTRAN_REAL16": 0,
              "OMPI_REAL16_MATCHES_C": 0, "HAVE_SHORT_FLOAT": 0, "HAVE_OPAL_SHORT_FLOAT_T": 0,
              "HAVE_SHORT_FLOAT__COMPLEX": 0, "HAVE_OPAL_SHORT_FLOAT_COMPLEX_T": 0})
    return c


def _cond(expr, cfg):
    e = expr.strip()
    e = re.sub(r"defined\s*\(\s*(\w+)\s*\)", lambda m: str(int(bool(cfg.get(m.group(1), 0)))), e)
    e = re.sub(r"[A-Za-z_]\w*", lambda m: str(int(cfg.get(m.group(0), 0))), e)
    return bool(eval(e.replace("&&", " and ").replace("||", " or ").replace("!", " not ")))  # noqa: S307


def _macros(text, cfg):
    """function-like #defines active under cfg (the file's #if nesting is flat)"""
    lines = text.replace("\\\n", " ").splitlines()
    macros, stack = {}, []
    for ln in lines:
        s = ln.strip()
        if s.startswith("#if"):
            stack.append(_cond(s[3:], cfg) if not s.startswith("#ifdef") and not s.startswith("#ifndef") else True)
        elif s.startswith("#else"):
            stack[-1] = not stack[-1]
        elif s.startswith("#endif"):
            stack.pop()
        elif s.startswith("#define") and all(stack):
            m = re.match(r"#define\s+(\w+)\((\w+)\s*,\s*(\w+)\)\s*(.*)", s)
            if m:
                macros[m.group(1)] = (m.group(2), m.group(3), re.sub(r"/\*.*?\*/", "", m.group(4)).strip())
    return macros


def _expand(expr, macros, depth=0):
    expr = expr.strip()
    m = re.fullmatch(r"(\w+)\((\w+)\s*,\s*(\w+)\)", expr)
    if not m or m.group(1) not in macros or depth > 8:
        return expr
    p1, p2, body = macros[m.group(1)]
    body = re.sub(r"\b" + p1 + r"\b", m.group(2), body)
    body = re.sub(r"\b" + p2 + r"\b", m.group(3), body)
    return body.replace("##", "")


def _entries(group_call, macros):
    """[OMPI_OP_BASE_TYPE_X] = value pairs of one group macro call"""
    out = {}
    body = _expand(group_call, macros)
    for part in re.split(r",\s*(?=\[|\w+\()", body):
        part = part.strip().rstrip(",")
        m = re.match(r"\[OMPI_OP_BASE_TYPE_(\w+)\]\s*=\s*(.+)", part)
        if m:
            val = _expand(m.group(2), macros)
            out[m.group(1)] = val if val != "NULL" else None
        elif re.fullmatch(r"\w+\(\w+\s*,\s*\w+\)", part):
            out.update(_entries(part, macros))       # nested group (FLOATING_POINT_FORTRAN_REAL)
    return out


def pattern(fortran, three=False):
    """{(op name, type slot name)} with a kernel in the reference table."""
    text = open(SRC).read()
    macros = _macros(text, config(fortran))
    table = "ompi_op_base_3buff_functions" if three else "ompi_op_base_functions"
    m = re.search(r"ompi_op_base_(?:3buff_)?handler_fn_t\s+" + table + r"\s*\[[^\]]*\]\s*\[[^\]]*\]\s*=\s*\{", text)
    assert m, table
    depth, i = 1, m.end()
    while depth:
        depth += {"{": 1, "}": -1}.get(text[i], 0)
        i += 1
    body = re.sub(r"/\*.*?\*/", "", text[m.end():i - 1], flags=re.S)
    pat = set()
    for row in re.finditer(r"\[OMPI_OP_BASE_FORTRAN_(\w+)\]\s*=\s*\{(.*?)\}", body, flags=re.S):
        op = row.group(1)
        for call in re.findall(r"\w+\(\w+\s*,\s*\w+\)", row.group(2)):
            for t, v in _entries(call, macros).items():
                if v:
                    pat.add((op, t))
    return pat


def available():
    return os.path.exists(SRC)
