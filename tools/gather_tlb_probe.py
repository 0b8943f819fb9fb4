#!/usr/bin/env python3
"""Random-row gather rate: 118k rows of 3 KB from a 10M x 768 fp32 array,
(a) uniformly random rows over the whole 30.7 GB, (b) the same count in 1000
windows of 256 consecutive rows (one IVF list each, list-ordered copy), (c)
random rows within the first 1 GB.  torch.index_select (a plain gather; the
ratios are what matter: page-walk cost of scattered rows)."""
import json
import torch

def main():
    n, d, m = 10_000_000, 768, 118_000
    torch.cuda.set_device(0)
    rows = torch.empty((n, d), dtype=torch.float32, device="cuda")
    rows.fill_(1.0)
    g = torch.Generator(device="cuda").manual_seed(1)
    arms = {
        "random_30GB": torch.randint(0, n, (m,), device="cuda", generator=g),
        "windows_256": (torch.randint(0, n // 256, (1000,), device="cuda", generator=g)[:, None] * 256
                        + torch.randint(0, 256, (1000, 118), device="cuda", generator=g)).reshape(-1),
        "random_1GB": torch.randint(0, 1 << 30 >> 12, (m,), device="cuda", generator=g),
    }
    out = torch.empty((m, d), dtype=torch.float32, device="cuda")
    for name, idx in arms.items():
        idx = idx[:m].contiguous()
        for _ in range(3):
            torch.index_select(rows, 0, idx, out=out)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        reps = 20
        for _ in range(reps):
            torch.index_select(rows, 0, idx, out=out)
        ev[1].record()
        torch.cuda.synchronize()
        ms = ev[0].elapsed_time(ev[1]) / reps
        print(json.dumps({"arm": name, "rows": int(idx.numel()), "ms": round(ms, 4),
                          "read_TBps": round(idx.numel() * d * 4 / ms / 1e9, 3)}), flush=True)

if __name__ == "__main__":
    main()
