#!/usr/bin/env python3
"""Effective shader clock under load (torch.cuda._sleep spins a known number of clock64() cycles)."""
import torch

a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
for phase in ("cold", "after-gemm-load"):
    if phase != "cold":
        for _ in range(50):
            a @ a
    for cyc in (10**6, 10**7):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        torch.cuda._sleep(cyc)
        e.record()
        e.synchronize()
        ms = s.elapsed_time(e)
        print(f"{phase}: _sleep({cyc}) {ms:.3f} ms -> {cyc / ms / 1e3:.0f} MHz (clock64 rate)")
s = torch.cuda.Event(enable_timing=True)
e = torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(20):
    a @ a
e.record()
e.synchronize()
ms = s.elapsed_time(e) / 20
print(f"8192^3 bf16 GEMM {ms:.3f} ms -> {2 * 8192**3 / ms / 1e9:.0f} TFLOP/s")
