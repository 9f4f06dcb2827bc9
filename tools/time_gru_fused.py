"""Time cn_gru_fwd_fused vs the unfused hipBLASLt addmm + cn_gru_fwd_step pair at C4's spatial-edge step
(B = 20,480 rows, H = 256) with HIP events: prints bench.gru_gemm_roofline's dict."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda:0")
    for B in (20480, 40960):
        print(json.dumps(bench.gru_gemm_roofline(torch, dev, B, 256, reps=100)), flush=True)
