"""The RCCL data path of mx_allreduce (MX_ALLREDUCE_RCCL, algorithm id 100).
bench.py's N>1 run times ncclAllReduce on its own RCCL communicator whenever
every rank has a GPU of its own (`rccl_leg`, checked against the oracle under
the reduction-order bound of `order_bound_check`, tests/test_bench_tolerance.py).

RCCL refuses two ranks on one GPU, and the test pool has one GPU per box, so
this covers what one GPU can: communicator creation with MX_COMM_RCCL
(ncclGetUniqueId / ncclCommInitRank over the host allgather), the type and op
mapping of every supported pair, the unsupported pairs failing loudly, and
the result of a one-rank ncclAllReduce (the input itself, bit for bit).
Results across ranks differ from the reference's fold order (RCCL's own
reduction order), which is why the path is never the default.
"""
import numpy as np
import pytest

import mxompi

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

SUPPORTED = [("FLOAT", "SUM"), ("FLOAT", "MAX"), ("DOUBLE", "PROD"), ("INT32_T", "MIN"), ("UINT8_T", "SUM"),
             ("INT64_T", "MAX"), ("UINT64_T", "SUM"), ("INT8_T", "MIN"), ("UINT32_T", "PROD"), ("REAL8", "SUM")]
UNSUPPORTED = [("LONG_DOUBLE", "SUM"), ("FLOAT_INT", "MAXLOC"), ("FLOAT", "BAND"), ("UINT16_T", "SUM")]


@pytest.fixture(scope="module")
def rccl_comm():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    torch.cuda.set_device(0)
    mxompi.init(0)
    comm = mxompi.Comm(0, 1, lambda b: [b], device=0, staging_bytes=4 << 20,
                       flags=mxompi.COMM_IPC | mxompi.COMM_RCCL)
    yield comm
    comm.close()


@pytest.mark.parametrize("t,op", SUPPORTED)
def test_rccl_allreduce_one_rank_returns_the_input(rccl_comm, t, op):
    es = mxompi.type_size(t)
    count = 1_000_003
    rng = np.random.default_rng(7)
    x = torch.from_numpy(rng.integers(0, 256, count * es, dtype=np.uint8)).to("cuda")
    if t in ("FLOAT", "DOUBLE", "REAL8"):   # finite values: NaN payloads are RCCL's business
        x = torch.from_numpy((rng.random(count) * 2 - 1).astype(np.float32 if t == "FLOAT" else np.float64)
                             .view(np.uint8)).to("cuda")
    out = torch.zeros_like(x)
    st = torch.cuda.current_stream().cuda_stream
    rccl_comm.allreduce(x.data_ptr(), out.data_ptr(), count, t, op, "rccl", st)
    torch.cuda.synchronize()
    assert torch.equal(out, x)


@pytest.mark.parametrize("t,op", UNSUPPORTED)
def test_rccl_unsupported_pairs_fail_loudly(rccl_comm, t, op):
    es = mxompi.type_size(t)
    x = torch.zeros(64 * es, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    with pytest.raises(mxompi.MxError):
        rccl_comm.allreduce(x.data_ptr(), x.data_ptr(), 64, t, op, "rccl", st)
