"""Drive pack + unpack of one golden vector type at ~1 GiB packed, for
rocprofv3 --pmc passes (HBM bytes of K5/K6 with gaps on the user side).
usage: python tools/pmc_unpack.py [type_name] [iters]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zhpe-ompi_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402
import golden_io  # noqa: E402
import mxompi as mx  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "vector_f32_b4_s8"
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    mx.init(0)
    _, recs = golden_io.ddt_records()
    rec = next(r for r in recs if r["name"] == name)
    dt = mx.Datatype(rec["desc"].tobytes(), rec["nrec"], rec["size"], rec["lb"], rec["ub"])
    count = (1 << 30) // rec["size"]
    ext = rec["ub"] - rec["lb"]
    span = ext * (count - 1) + rec["true_ub"] - rec["true_lb"]
    U = torch.randint(0, 256, (span,), dtype=torch.uint8, device="cuda")
    P = torch.empty(count * rec["size"], dtype=torch.uint8, device="cuda")
    sp = torch.cuda.current_stream().cuda_stream
    base = U.data_ptr() - rec["true_lb"]
    for _ in range(iters):
        dt.pack(count, base, P.data_ptr(), stream=sp)
        dt.unpack(count, base, P.data_ptr(), stream=sp)
    torch.cuda.synchronize()
    print(f"{name}: packed {count * rec['size']} B per call, user span {span} B, {iters} pack+unpack")


if __name__ == "__main__":
    main()
