"""Calibration only (not product code): the vendor library's rate (torch.matmul
-> hipBLASLt / rocBLAS) on the learner's GEMM shapes, beside which the twin
GEMM's isolated numbers (tools/gemmh_bench) can be read.  fp32 with TF32 off
(exact fp32 products, the C3 accuracy class), bf16 for C5.
  python tools/gpu/vendor_gemm_ref.py > gpurun_out/vendor_gemm.txt"""
import torch

torch.backends.cuda.matmul.allow_tf32 = False
torch.backends.cudnn.allow_tf32 = False
dev = "cuda"
shapes = [  # (label, M, N, K, dtype)
    ("c3 fwd", 4096, 1024, 1024, torch.float32),
    ("c3 fwd K=2048", 4096, 1024, 2048, torch.float32),
    ("c3 dx", 4096, 2048, 1024, torch.float32),
    ("c3 wgrad", 2048, 1024, 4096, torch.float32),
    ("c5 first fwd", 4096, 2048, 384, torch.bfloat16),
    ("c5 fwd", 4096, 2048, 2048, torch.bfloat16),
    ("c5 fwd K=4096", 4096, 2048, 4096, torch.bfloat16),
    ("c5 dx", 4096, 4096, 2048, torch.bfloat16),
    ("c5 wgrad", 4096, 2048, 4096, torch.bfloat16),
]
for label, M, N, K, dt in shapes:
    a = torch.rand(M, K, device=dev, dtype=dt) - 0.5
    b = torch.rand(K, N, device=dev, dtype=dt) - 0.5
    for _ in range(5):
        c = a @ b
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            c = a @ b
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / 20 * 1e3)
    tf = 2.0 * M * N * K / (best * 1e-6) / 1e12
    print("%-16s %-9s M=%d N=%d K=%d  %8.2f us  %7.1f TF" % (label, str(dt).split(".")[1], M, N, K,
                                                               best, tf), flush=True)
