"""Cost of one 32x32 block of the split-bf16 row-GEMM chain (K = 128) per wave, by form
(gine_probe_chain): shader-clock ticks per block, median over waves, at 1 and 2 workgroups
per CU.  Ideal: 48 v_mfma_f32_32x32x16_bf16 x 32 cycles = 1,536 per block.
    python tools/chain_micro.py [--reps 64]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "raincast-gnn_amd"))
import torch  # noqa: E402

from raincast_gnn import _lib  # noqa: E402

FORMS = {0: "split in loop", 1: "pre-split planes", 2: "MFMA only", 3: "two chains interleaved",
         4: "split pipelined"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=64)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    s = _lib.stream_handle(dev)
    for blocks in (cus, 2 * cus):
        sink = torch.empty(blocks * 256, device=dev)
        ticks = torch.zeros(blocks * 4, dtype=torch.int64, device=dev)
        for v, name in FORMS.items():
            for _ in range(2):
                _lib.call("gine_probe_chain", v, a.reps, blocks, _lib.ptr(sink), _lib.ptr(ticks), s)
            torch.cuda.synchronize()
            per = ticks.double() / a.reps / (2 if v == 3 else 1)
            print(f"{blocks // cus} wg/CU  form {v} ({name:22s}): {per.median().item():7.0f} "
                  f"ticks per 32x32 block (p90 {per.quantile(0.9).item():.0f})", flush=True)


if __name__ == "__main__":
    main()
