"""Time sc_scan_exclusive_i32 at 2^28 under the current SC_* environment (tuning helper)."""
import os
import sys

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from cuda_pathtracer_amd._native import check_sc, lib  # noqa: E402

n = int(os.environ.get("N", 1 << 28))
dev = torch.device("cuda", 0)
op = os.environ.get("OP", "scan")
a = torch.randint(0, 50 if op == "scan" else 4, (n,), dtype=torch.int32, device=dev)
out = torch.empty_like(a)
cnt = torch.zeros(1, dtype=torch.int64, device=dev)
ws = torch.empty(int(lib().sc_workspace_bytes(n)), dtype=torch.uint8, device=dev)
st = torch.cuda.current_stream()


def call():
    if op == "scan":
        check_sc(lib().sc_scan_exclusive_i32(a.data_ptr(), out.data_ptr(), n, ws.data_ptr(), st.cuda_stream))
    elif op == "partition":
        check_sc(lib().sc_partition_i32(a.data_ptr(), out.data_ptr(), n, cnt.data_ptr(), ws.data_ptr(), st.cuda_stream))
    else:
        check_sc(lib().sc_compact_i32(a.data_ptr(), out.data_ptr(), n, cnt.data_ptr(), ws.data_ptr(), st.cuda_stream))


for _ in range(3):
    call()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
reps = 20
e0.record(st)
for _ in range(reps):
    call()
e1.record(st)
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / reps
if op == "scan":
    ok = bool(torch.equal(out[1:] - out[:-1], a[:-1])) and int(out[0].item()) == 0
    nbytes = 8 * n
elif op == "partition":
    idx = torch.arange(n, dtype=torch.int32, device=dev)
    live = idx[a != 0]
    ok = int(cnt.item()) == live.numel() and bool(torch.equal(out, torch.cat([live, idx[a == 0]])))
    nbytes = 8 * n
else:
    kept = a[a != 0]
    ok = int(cnt.item()) == kept.numel() and bool(torch.equal(out[:kept.numel()], kept))
    nbytes = 4 * n + 4 * kept.numel()
extra = ""
if int(os.environ.get("SC_EXPERIMENT", "0")) & 16:
    c = ws[:16].view(torch.int32).cpu().tolist()
    extra = f" lookbacks={c[2]} extra_rounds={c[3]} ({c[3] / max(c[2], 1):.2f}/lookback, last call)"
print(f"{os.environ.get('TAG','')} {op} ms={ms:.4f} GB/s={nbytes/ms/1e6:.0f} ok={ok}{extra}", flush=True)
