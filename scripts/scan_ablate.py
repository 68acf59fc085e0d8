"""Time sc_scan_exclusive_i32 at 2^28 under the current SC_* environment (tuning helper)."""
import os
import sys

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from cuda_pathtracer_amd._native import check_sc, lib  # noqa: E402

n = int(os.environ.get("N", 1 << 28))
dev = torch.device("cuda", 0)
a = torch.randint(0, 50, (n,), dtype=torch.int32, device=dev)
out = torch.empty_like(a)
ws = torch.empty(int(lib().sc_workspace_bytes(n)), dtype=torch.uint8, device=dev)
st = torch.cuda.current_stream()
for _ in range(3):
    check_sc(lib().sc_scan_exclusive_i32(a.data_ptr(), out.data_ptr(), n, ws.data_ptr(), st.cuda_stream))
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
reps = 20
e0.record(st)
for _ in range(reps):
    check_sc(lib().sc_scan_exclusive_i32(a.data_ptr(), out.data_ptr(), n, ws.data_ptr(), st.cuda_stream))
e1.record(st)
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / reps
ok = bool(torch.equal(out[1:] - out[:-1], a[:-1])) and int(out[0].item()) == 0
extra = ""
if int(os.environ.get("SC_EXPERIMENT", "0")) & 16:
    c = ws[:16].view(torch.int32).cpu().tolist()
    extra = f" lookbacks={c[2]} extra_rounds={c[3]} ({c[3] / max(c[2], 1):.2f}/lookback, last call)"
print(f"{os.environ.get('TAG','')} ms={ms:.4f} GB/s={8*n/ms/1e6:.0f} ok={ok}{extra}", flush=True)
