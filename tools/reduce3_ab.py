"""3-buffer reduce throughput of padded element types (diagnostic): HIP
events around 10 launches, 1 GiB per buffer.  A/B: MX_REDUCE_W32T=0|1."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zhpe-ompi_amd"))
import torch  # noqa: E402
import mxompi  # noqa: E402

mxompi.init(0)
nb = 1 << 30
for op, t in [("MAXLOC", "DOUBLE_INT"), ("MINLOC", "SHORT_INT"), ("SUM", "LONG_DOUBLE"),
              ("MAXLOC", "LONG_DOUBLE_INT"), ("SUM", "C_LONG_DOUBLE_COMPLEX"), ("SUM", "FLOAT")]:
    es = mxompi.type_size(t)
    n = nb // es
    a = torch.zeros(nb, dtype=torch.uint8, device="cuda")
    b = torch.zeros(nb, dtype=torch.uint8, device="cuda")
    o = torch.zeros(nb, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    mxompi.reduce3(op, t, a.data_ptr(), b.data_ptr(), o.data_ptr(), n, s.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(10):
        mxompi.reduce3(op, t, a.data_ptr(), b.data_ptr(), o.data_ptr(), n, s.cuda_stream)
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"MX_REDUCE_W32T={os.environ.get('MX_REDUCE_W32T', '1')} 3-buffer {op} {t}: {ms:.3f} ms "
          f"{3 * nb / ms / 1e6:.0f} GB/s (algorithmic 3 x 1 GiB)", flush=True)
    del a, b, o
