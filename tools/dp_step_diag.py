import os, sys, subprocess, socket, torch
ROOT = "/root/repo" if os.path.exists("/root/repo") else os.getcwd()
def port():
    s = socket.socket(); s.bind(("127.0.0.1", 0)); p = s.getsockname()[1]; s.close(); return p
os.environ["DS2_DP_GEOM"] = "config5"
for pairs in sys.argv[1].split(","):
    out = "/tmp/dpd_%s" % pairs
    env = dict(os.environ, PYTHONPATH=ROOT, DS2_DIST_BACKEND="gloo", DS2_DEVICE_INDEX="0", OMP_NUM_THREADS="2",
               DS2_DP_GEOM="config5", DS2_FP8_PAIRS=pairs)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(port()), os.path.join(ROOT, "tests", "dp_gpu_worker.py"), out]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    print("pairs", pairs, "rc", r.returncode, r.stderr[-500:] if r.returncode else "")
    g = [torch.load("%s.%d" % (out, k), weights_only=True) for k in range(2)]
    for k in range(2):
        for key in ("local", "dp", "step_local", "w_step", "ema_step"):
            bad = ~torch.isfinite(g[k][key])
            if bad.any():
                print("   rank", k, key, "non-finite", int(bad.sum()))
    d = (g[0]["w_step"] - g[1]["w_step"]).abs()
    print("pairs", pairs, "w_step equal", torch.equal(g[0]["w_step"], g[1]["w_step"]), "ndiff", int((d > 0).sum()), "max", float(d.max()))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import dp_gpu_worker as W
    from deepspeech_amd.trainer import Trainer, LRSchedule
    tr = Trainer(W.model(torch.device("cuda")), LRSchedule(1e-3, 10, 0.9))
    for name, (o, n) in zip(tr.arena.names, tr.arena.offsets):
        dd = d[o:o + n]
        nf = [int((~torch.isfinite(g[k]["w_step"][o:o + n])).sum()) for k in range(2)]
        nfg = [int((~torch.isfinite(g[k]["dp"][o:o + n])).sum()) for k in range(2)]
        nfl = [int((~torch.isfinite(g[k]["local"][o:o + n])).sum()) for k in range(2)]
        if (dd > 0).any() or any(nf) or any(nfg) or any(nfl):
            print("   ", name, "diff", int((dd > 0).sum()), "of", n, "nonfinite w", nf, "dp", nfg, "local", nfl)
