"""Time wh_mlp_forward (SAC policy forward, argmax) on B=65536 envs' agent rows per variant.
Prints us/launch and dense bf16 TFLOP/s (2 * rows * (in*h0 + h0*h1 + h1*9))."""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rllib-warehouse_amd")]
import torch  # noqa: E402
import warehouse  # noqa: E402
import warehouse.policy as wp  # noqa: E402

B = int(os.environ.get("MLP_B", 65536))
VARIANTS = os.environ.get("MLP_VARIANTS", "small,medium,large").split(",")
for abl, variant, na in [(a, v, n) for a in os.environ.get("MLP_ABLATE", "0").split(",")
                         for v, n in (("small", 4), ("medium", 8), ("large", 16)) if v in VARIANTS]:
    os.environ["WH_MLP_ABLATE"] = abl
    net = wp.MLPPolicy(variant, seed=1)
    rows = B * na
    x = torch.randn((rows, net.in_dim), device="cuda") * 4
    acts = torch.empty(rows, dtype=torch.int32, device="cuda")
    if os.environ.get("MLP_X") == "1":
        # the fragment-order operand (wh_observe_x's layout): random bf16 of magnitude [0.5, 1)
        kq = (net.in_dim + 2 + 15) // 16
        bits = torch.randint(0, 1 << 15, ((rows + 31) // 32, kq, 64, 8), device="cuda", dtype=torch.int32)
        xf = ((bits & 0x807F) | 0x3F00).to(torch.int16).view(torch.uint8).contiguous()
        fwd = lambda: net.forward_x(xf, rows, actions=acts, step=0)   # noqa: E731
    else:
        fwd = lambda: net(x, actions=acts, step=0)   # noqa: E731
    for _ in range(3):
        fwd()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 10
    t0.record()
    for _ in range(reps):
        fwd()
    t1.record()
    torch.cuda.synchronize()
    us = t0.elapsed_time(t1) / reps * 1e3
    h0, h1 = net.hidden
    flop = 2.0 * rows * (net.in_dim * h0 + h0 * h1 + h1 * 9)
    print(f"ablate={abl} {variant:6s} rows={rows:8d} [{net.in_dim},{h0},{h1},9] {us:9.1f} us  {flop / us / 1e6:7.1f} TFLOP/s",
          flush=True)
    if os.environ.get("MLP_LIB") == "1":
        # the same network through the vendor library (torch bf16 linear = hipBLASLt GEMMs, unfused
        # bias/ReLU/argmax): what a library route reaches on these shapes, on the same box
        g = torch.Generator(device="cpu").manual_seed(1)
        dims = [net.in_dim, h0, h1, 9]
        ws = [(torch.randn(dims[i + 1], dims[i], generator=g) / dims[i] ** 0.5).to("cuda", torch.bfloat16)
              for i in range(3)]
        bs = [torch.zeros(dims[i + 1], device="cuda", dtype=torch.bfloat16) for i in range(3)]
        xb = x.to(torch.bfloat16)
        f = torch.nn.functional

        def lib_fwd():
            h = f.relu(f.linear(xb, ws[0], bs[0]))
            h = f.relu(f.linear(h, ws[1], bs[1]))
            return f.linear(h, ws[2], bs[2]).argmax(dim=1)

        def timed(fn, n=10):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            t0.record()
            for _ in range(n):
                fn()
            t1.record()
            torch.cuda.synchronize()
            return t0.elapsed_time(t1) / n * 1e3

        us_chain = timed(lib_fwd)
        h0t = torch.randn(rows, h0, device="cuda").to(torch.bfloat16)
        us_g0 = timed(lambda: torch.matmul(xb, ws[0].t()))
        us_g1 = timed(lambda: torch.matmul(h0t, ws[1].t()))
        print(f"   library {variant:6s} chain {us_chain:9.1f} us {flop / us_chain / 1e6:7.1f} TFLOP/s | "
              f"GEMM0 [{rows}x{dims[0]}]x[{dims[0]}x{h0}] {2 * rows * dims[0] * h0 / us_g0 / 1e6:7.1f} TFLOP/s | "
              f"GEMM1 [{rows}x{h0}]x[{h0}x{h1}] {2 * rows * h0 * h1 / us_g1 / 1e6:7.1f} TFLOP/s", flush=True)
