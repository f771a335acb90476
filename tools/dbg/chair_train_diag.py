"""Diagnostic: train.py's loop on the chair (HIP drop-ins, DataParallelTrainer in one process) with
loss / train-view PSNR / P traces, for several variants.  Usage: python tools/dbg/chair_train_diag.py"""
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "gaussian-splatting-npu_amd"), os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import test_chair_train as t  # noqa: E402


def run(variant, iters=3000, res=800):
    import diff_gaussian_rasterization as dgr
    from diff_gaussian_rasterization import multiview
    train, test, raw0, extent, P0 = t._load(res)
    dev = torch.device("cuda:0")
    opt = "adam" if variant.get("adam") else "sparse_adam"
    trainer = multiview.DataParallelTrainer({k: v.to(dev) for k, v in raw0.items()}, optimizer=opt,
                                            spatial_lr_scale=extent, seed=0)
    def views(d):
        out = []
        for v in train:
            gt = v.original_image.to(dev)
            ex = {} if variant.get("nomask") else {"alpha_mask": v.alpha_mask.to(dev)}
            if variant.get("nomask"):
                gt = gt * v.alpha_mask.to(dev)
            out.append((t._settings(dgr, v, d), gt, ex))
        return out
    vb = {d: views(d) for d in range(4)}
    order = random.Random(0)
    stack, log = [], []
    losses = []
    t0 = time.time()
    for it in range(1, iters + 1):
        degree = min(it // 1000, 3)
        if not stack:
            stack = list(range(len(train)))
        vi = stack.pop(order.randint(0, len(stack) - 1))
        l, did = trainer.iteration(it, [vb[degree][vi]], extent)
        losses.append(float(l[0]))
        if it % 500 == 0:
            with torch.no_grad():
                act = t._activate(trainer.params)
                ftr, mtr = t._hip_test_psnrs(dgr, act, train[:6], degree)
                fte, mte = t._hip_test_psnrs(dgr, act, test, degree)
                op = torch.sigmoid(trainer.params["opacity"]).mean().item()
            log.append({"it": it, "loss": round(float(np.mean(losses[-100:])), 5), "P": int(trainer.P),
                        "train_masked": round(float(mtr.mean()), 3), "test_masked": round(float(mte.mean()), 3),
                        "test_full": round(float(fte.mean()), 3), "mean_opacity": round(op, 4),
                        "s": round(time.time() - t0, 1)})
            print(variant, log[-1], flush=True)
    return log


if __name__ == "__main__":
    out = {}
    for name, v in (("sparse_adam", {}), ("adam", {"adam": True}), ("nomask_black", {"nomask": True})):
        out[name] = run(v)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "chair_train_diag.json"), "w"), indent=1)
