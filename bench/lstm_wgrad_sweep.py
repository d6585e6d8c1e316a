"""Tile / split-K sweep of the LSTM kernel-gradient GEMM (fp32, M=157 [x,h,1] rows, N=512 gates,
K=T*B=3584): dK = [x_t, h_{t-1}, 1]^T . dgates over every timestep and batch row."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import dtfe  # noqa: F401
from dtfe import ops

dev = torch.device("cuda", 0)
T, B, I, H = 28, 128, 28, 128
xh = torch.randn(T, B, I + H, device=dev)
dg = torch.randn(T, B, 4 * H, device=dev)
gK = torch.empty(I + H, 4 * H, device=dev)
gb = torch.empty(4 * H, device=dev)
ref = torch.cat([xh.reshape(-1, I + H), torch.ones(T * B, 1, device=dev)], 1).double().t() @ dg.reshape(-1, 4 * H).double()
for tile, splits in [(None, 1), (13, 1), (4, 1), (4, 4), (4, 8), (4, 16), (0, 1), (0, 4), (0, 8), (0, 16), (2, 8), (3, 8)]:
    def run():
        kw = {} if tile is None else dict(tile=tile, splits=splits)
        ops.gemm(xh, dg, gK, M=I + H + 1, N=4 * H, K=T * B, amode=ops.RMAJ, lda=I + H, bmode=ops.RMAJ, ldb=4 * H,
                 a_ones_row=I + H, bias_out=gb, **kw)
    try:
        run()
    except Exception as e:  # noqa: BLE001
        print(tile, splits, "error", str(e)[:80]); continue
    torch.cuda.synchronize()
    err = max((gK.double() - ref[:-1]).abs().max().item(), (gb.double() - ref[-1]).abs().max().item())
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(5): run()
    s.record()
    for _ in range(50): run()
    e.record(); torch.cuda.synchronize()
    print("tile", tile, "splits", splits, "us %.1f" % (s.elapsed_time(e) / 50 * 1e3), "maxerr %.2e" % err, flush=True)

for splits in (8, 16, 32, 56, 112):
    ws = torch.empty(ops.tallk_ws_floats(I + H, 4 * H, splits), device=dev)
    def run():
        ops.wgrad_tallk(xh, I + H, dg, 4 * H, I + H, 4 * H, T * B, gK, bias=gb, splits=splits, workspace=ws)
    run(); torch.cuda.synchronize()
    err = max((gK.double() - ref[:-1]).abs().max().item(), (gb.double() - ref[-1]).abs().max().item())
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(5): run()
    s.record()
    for _ in range(50): run()
    e.record(); torch.cuda.synchronize()
    print("tallk splits", splits, "us %.1f" % (s.elapsed_time(e) / 50 * 1e3), "maxerr %.2e" % err, flush=True)
