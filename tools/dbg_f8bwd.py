import sys, torch
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
from deepspeech_amd.ops import rnn as RNN
import test_kernels_gpu as K
cuda = torch.device("cuda")
N, H, ndir, T = 8, 256, 1, 2
P = H // 64
plan = RNN.plan_for(N, H, "gru", ndir, cuda)
torch.manual_seed(1)
gx = (torch.randn(T, N, 3 * H, device=cuda) * 0.5).to(torch.bfloat16)
lens = torch.full((N,), T, device=cuda, dtype=torch.int32)
U = [(torch.randn(3 * H, H, device=cuda) * (1.5 / H ** 0.5)).to(torch.bfloat16)]
bh = [torch.randn(3 * H, device=cuda) * 0.1]
y, (hx, hs, gates) = RNN._run_fwd_fp8(gx, lens, U, bh + [None], plan)
dy = torch.randn(T, N, H, device=cuda).to(torch.bfloat16)
BG = 8 // ndir; R = -(-N // BG)
dbg = torch.zeros(BG * P * 8 * H + BG * P * 8 * 3 * 64, device=cuda)
dgx, dgh, parts = RNN._run_bwd_fp8(dy, lens, U + [None], hs, gates, plan, 3 * H, dbg=dbg)
part = dbg[:BG * P * 8 * H].view(BG, P, 8, H)
torch.cuda.synchronize(); RNN.check_errors()
ghv = dgh[0, T - 1, :N].float()             # [N, 3H] exact bf16 gate grads of step T-1
u = U[0].float()
uq = K._e4m3_pow2(u, u.abs().max())
for mem in range(P):
    cols = torch.cat([torch.arange(g * H + 64 * mem, g * H + 64 * mem + 64) for g in range(3)]).to(cuda)
    gv = ghv[:, cols]
    am = gv.abs().amax(1, keepdim=True)
    q = K._e4m3_pow2(gv, am)
    want = q @ uq[cols]                         # [N, H]
    got = torch.stack([part[b // R, mem, b % R] for b in range(N)])
    print("mem %d rel %.4f |want| %.3e |got| %.3e ratio %.4f" % (mem, K._rel(got, want), want.norm(), got.norm(),
                                                                 float(got.norm() / want.norm())))
    for g in range(3):
        cg = cols[64 * g:64 * (g + 1)]
        wg = K._e4m3_pow2(ghv[:, cg], am) @ uq[cg]
        print("   gate %d alone: rel(got, gate part) %.4f" % (g, K._rel(got, wg)))
# consumer side at s = T-2: dhrec as the kernel summed it, vs the sum of the dumped partials
off = BG * P * 8 * H
cons = dbg.view(-1)[off:off + BG * P * 8 * 3 * 64].view(BG, P, 8, 3, 64)
for mem in range(P):
    got = torch.stack([cons[b // R, mem, b % R, 0] for b in range(N)])            # [N, 64]
    summed = sum(torch.stack([part[b // R, j, b % R, 64 * mem:64 * mem + 64] for b in range(N)]) for j in range(P))
    dyv = torch.stack([cons[b // R, mem, b % R, 1] for b in range(N)])
    car = torch.stack([cons[b // R, mem, b % R, 2] for b in range(N)])
    print("consumer mem %d: rel(kernel dhrec, sum of partials) %.4f |dhrec| %.3e |sum| %.3e |dy| %.3e |carry| %.3e" % (
        mem, K._rel(got, summed), got.norm(), summed.norm(), dyv.norm(), car.norm()))
full = q_all = None
ghv1 = dgh[0, T - 1, :N].float()
blk1 = ghv1.view(N, 3, P, 64).abs().amax(dim=(1, 3))
am1 = blk1[:, None, :, None].expand(N, 3, P, 64).reshape(N, 3 * H)
full = K._e4m3_pow2(ghv1, am1) @ uq
car_py = dy[1].float() * gates[0, 1, :N, :, 1].float()
for mem in range(P):
    sl = slice(64 * mem, 64 * mem + 64)
    gk = torch.stack([cons[b // R, mem, b % R, 0] for b in range(N)])
    dyk = torch.stack([cons[b // R, mem, b % R, 1] for b in range(N)])
    ck = torch.stack([cons[b // R, mem, b % R, 2] for b in range(N)])
    print("mem %d: rel dhrec %.4f dy %.4f carry %.4f" % (mem, K._rel(gk, full[:, sl]), K._rel(dyk, dy[0].float()[:, sl]),
                                                      K._rel(ck, car_py[:, sl])))
g0 = gates[0, 0, :N].float(); hp0 = hs[0, 0, :N].float()
for mem in range(P):
    sl = slice(64 * mem, 64 * mem + 64)
    dhk = torch.stack([cons[b // R, mem, b % R, 0] + cons[b // R, mem, b % R, 1] + cons[b // R, mem, b % R, 2]
                       for b in range(N)])
    r, z, n, ghn = g0[:, sl, 0], g0[:, sl, 1], g0[:, sl, 2], g0[:, sl, 3]
    dn = dhk * (1 - z); dz = dhk * (hp0[:, sl] - n); dan = dn * (1 - n * n); dr = dan * ghn
    want = [dr * r * (1 - r), dz * z * (1 - z), dan]
    for g in range(3):
        got = dgx[0, :, g * H + 64 * mem:g * H + 64 * mem + 64].float()
        print("mem %d gate %d rel(dgx kernel, cell(kernel dh)) %.4f |got| %.3e |want| %.3e" % (
            mem, g, K._rel(got, want[g]), got.norm(), want[g].norm()))
