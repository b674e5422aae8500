"""CPU: the op oracle restatement against the committed vectors and the
reference's table text.

* The (op, type) availability pattern of both table variants (C only: 116
  pairs, with Fortran: 176) is read from the text of the reference's
  op_base_functions.c (tests/ref_optable.py expands its group macros and
  designated initialisers) and must equal the restatement's.
* The golden vectors (tests/golden/op_vectors.bin, oracle/gen_op_golden.c)
  are regression vectors of the restatement; the reference holds no known
  answers for these kernels, so op-kernel VALUES are
  unpinned.
"""
import ctypes

import numpy as np
import pytest

import golden_io
import oracle_lib
import ref_optable

RECS = golden_io.op_records()


def test_golden_covers_all_176_pairs():
    pairs2 = {(r["op"], r["type"]) for r in RECS if r["kind"] == 2}
    pairs3 = {(r["op"], r["type"]) for r in RECS if r["kind"] == 3}
    assert len(pairs2) == 176 and pairs2 == pairs3


@pytest.mark.parametrize("fortran", [0, 1])
def test_pattern_matches_reference_tables(fortran):
    import mxompi
    O = oracle_lib.oracle()
    mine = {(mxompi.OPS[op], mxompi.TYPES[t]) for op in range(15) for t in range(41)
            if O.mxo_supported(op, t, fortran)}
    assert len(mine) == (176 if fortran else 116)
    if not ref_optable.available():
        pytest.skip("reference source not present")
    for three in (False, True):
        assert mine == ref_optable.pattern(fortran, three)


@pytest.mark.parametrize("rec", RECS, ids=lambda r: f"k{r['kind']}-op{r['op']}-t{r['type']}")
def test_oracle_matches_golden(rec):
    O = oracle_lib.oracle()
    a = rec["a"].copy()
    b = rec["b"].copy()
    if rec["kind"] == 2:
        rc = O.mxo_reduce2(rec["op"], rec["type"], a.ctypes.data, b.ctypes.data, rec["n"], 1)
        out = b
    else:
        out = np.zeros_like(b)
        rc = O.mxo_reduce3(rec["op"], rec["type"], a.ctypes.data, b.ctypes.data,
                           out.ctypes.data, rec["n"], 1)
    assert rc == 0
    golden_io.assert_op_equal(out, rec["out"], rec["op"], rec["type"])
