"""Drive pack + unpack of one datatype at ~1 GiB packed, for rocprofv3 --pmc
passes (HBM bytes of K5/K6 with gaps on the user side).
Types as tools/conv_probe.py names them (golden names, vec:..., tri:n, idx:n:seed).
usage: python tools/pmc_unpack.py [type_name] [iters]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zhpe-ompi_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402
import mxompi as mx  # noqa: E402
import conv_probe  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "vector_f32_b4_s8"
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    mx.init(0)
    dt, size, ext, tlb, tub = conv_probe.make_type(mx, name)
    count = (1 << 30) // size
    span = ext * (count - 1) + tub - tlb
    U = torch.randint(0, 256, (span,), dtype=torch.uint8, device="cuda")
    P = torch.empty(count * size, dtype=torch.uint8, device="cuda")
    sp = torch.cuda.current_stream().cuda_stream
    base = U.data_ptr() - tlb
    for _ in range(iters):
        dt.pack(count, base, P.data_ptr(), stream=sp)
        dt.unpack(count, base, P.data_ptr(), stream=sp)
    torch.cuda.synchronize()
    print(f"{name}: packed {count * size} B per call, user span {span} B, {iters} pack+unpack, path {dt.last_path}")


if __name__ == "__main__":
    main()
