"""Developer probe: how much the distillation step's two forwards overlap.  Builds bench.py's C5 step as a
hiseg.GraphedBranchStep, then times (HIP events on the caller's stream, median of 20) the teacher graph alone, the
student graph alone, the tail graph alone, both forward graphs launched side by side, and the whole step.
Usage: python tools/distill_branches.py [--unfrozen N]"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "human-instance-segmentation_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden"))


def main():
    import filler
    import hiseg
    from hiseg.streams import role_stream
    unfrozen = int(sys.argv[sys.argv.index("--unfrozen") + 1]) if "--unfrozen" in sys.argv else 0
    dev = torch.device("cuda:0")
    model, loss_fn = hiseg.create_unet_distillation_model("timm-efficientnet-b0", "timm-efficientnet-b7",
                                                          teacher_checkpoint="absent.pth", device="cpu",
                                                          progressive_unfreeze=True)
    filler.fill_module(model.student, seed=11)
    filler.fill_module(model.teacher, seed=12)
    hiseg.set_compute_dtype(model, torch.bfloat16)
    model = model.to(dev).train()
    loss_fn.temperature = 4.0
    b, hw = 4, 640
    x = torch.randn(b, 3, hw, hw, generator=torch.Generator().manual_seed(100)).to(dev)
    m = (torch.rand(b, 1, hw, hw, generator=torch.Generator().manual_seed(1)) > 0.5).float().to(dev)
    enc = model.unfreeze_encoder_blocks(unfrozen, learning_rate_scale=0.1) if unfrozen else None
    st, fwd = {"opt": None, "enc": None}, {}

    def tail():
        loss, _ = loss_fn(fwd["s"], fwd["t"], m)
        if st["opt"] is None:
            st["opt"] = hiseg.FusedAdamW(model.student, lr=1e-4, weight_decay=1e-4, max_grad_norm=1.0,
                                         params=model.student.get_decoder_parameters())
            if enc:
                st["enc"] = hiseg.FusedAdamW(model.student, lr=1e-5, weight_decay=1e-4, max_grad_norm=None,
                                             params=enc)
        opts = [o for o in (st["opt"], st["enc"]) if o is not None]
        for o in opts:
            o.zero_grad()
        loss.backward()
        for o in opts:
            o.step()
        return loss

    def teacher():
        fwd["t"] = model.teacher(x)

    def student():
        fwd["s"] = model.student(x)

    run = hiseg.GraphedBranchStep(teacher, student, tail, lambda: st["opt"])
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    gb, gh, gt = run.graphs
    side = role_stream("teacher")
    main = torch.cuda.current_stream()

    def both():
        side.wait_stream(main)
        with torch.cuda.stream(side):
            gb.replay()
        gh.replay()
        main.wait_stream(side)

    def timed(fn, n=20):
        ts = []
        for _ in range(n):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return round(statistics.median(ts), 3)

    res = {"teacher": timed(gb.replay), "student": timed(gh.replay), "tail": timed(gt.replay),
           "both_forwards": timed(both), "step": timed(run),
           "step_back_to_back": round(timed(lambda: [run() for _ in range(10)], 5) / 10, 3)}
    print(res, flush=True)


if __name__ == "__main__":
    main()
