import sys, torch
sys.path.insert(0, "/root/repo")
sys.argv = ["bench.py"]
import bench
args = bench.parse()
dev = torch.device("cuda")
pair, opt, loss_fn, it, step_fn, tr, te = bench.setup(args, dev)
flat = opt.flat
print("inactive params:", list(flat._inactive.keys()), "restrict_version", flat.restrict_version)
for _ in range(3):
    b, a = next(it)
    step_fn(b, a, loss_fn, opt)
torch.cuda.synchronize()
print("after steps inactive:", list(flat._inactive.keys()), "restrict_version", flat.restrict_version,
      "ok_version", getattr(opt, "_restrict_ok_version", None))
tab, n = flat.span_table()
print("spans", n, "active elems", int(tab[:, 2].sum()) * 4, "of", flat.numel)
