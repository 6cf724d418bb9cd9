"""Where the input-inclusive (H2D) leg of bench.py loses time at config 2: the same train step fed four ways.
  hbm      : device-resident fp32 clips (bench.py's timed leg)
  convert  : device-resident u8 clips, u8 -> fp32 on the device each step (no copy)
  copy     : pinned host u8 -> device copy on the copy stream each step, the step still reads resident fp32 clips
  h2d      : ClipStager (copy + convert, bench.py's h2d_inclusive leg)
Prints one JSON line of ms/step per variant (usage: python tools/h2d_probe.py [steps])."""
import json, sys, time

import torch

sys.path.insert(0, ".")
import vad_amd._native as nat  # noqa: E402
from vad_amd.cad import CausalAnomalyDetector  # noqa: E402
from vad_amd.data import ClipStager  # noqa: E402
from vad_amd.train import CadTrainer, apply_memory_efficient_training  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = CausalAnomalyDetector()
    apply_memory_efficient_training(model)
    model = model.to(dev)
    tr = CadTrainer(model, lr=3e-4, seed=1234)
    B, T, H, W = 8, 16, 227, 227
    labels = torch.tensor([b % 2 for b in range(B)], dtype=torch.int64, device=dev)
    u8h = [torch.randint(0, 256, (B, T, 1, H, W), dtype=torch.uint8).pin_memory() for _ in range(2)]
    u8d = [u.to(dev) for u in u8h]
    pool = [torch.empty(B, T, 1, H, W, device=dev) for _ in range(2)]
    for k in range(2):
        nat.check(nat.lib().vad_u8_to_clip(u8d[k].data_ptr(), u8d[k].numel(), 0, pool[k].data_ptr(), nat.stream_of(dev)))
    copy_stream = torch.cuda.Stream(dev)
    scratch = [torch.empty_like(u8d[0]) for _ in range(2)]
    stager = ClipStager(dev, mode=0)
    out = {}

    def run(name, body):
        for i in range(3):
            body(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            body(i)
        torch.cuda.synchronize()
        out[name] = round(1e3 * (time.perf_counter() - t0) / steps, 4)

    run("hbm", lambda i: tr.step(pool[i % 2], labels))

    def convert(i):
        x = torch.empty(B, T, 1, H, W, device=dev)
        nat.check(nat.lib().vad_u8_to_clip(u8d[i % 2].data_ptr(), u8d[i % 2].numel(), 0, x.data_ptr(), nat.stream_of(dev)))
        tr.step(x, labels)
    run("convert", convert)

    def copy(i):
        copy_stream.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(copy_stream):
            scratch[i % 2].copy_(u8h[i % 2], non_blocking=True)
        tr.step(pool[i % 2], labels)
    run("copy", copy)

    state = {"h": stager.issue(u8h[0])}

    def h2d(i):
        x = stager.finish(state["h"])
        state["h"] = stager.issue(u8h[(i + 1) % 2])
        tr.step(x, labels)
    run("h2d", h2d)
    run("hbm_again", lambda i: tr.step(pool[i % 2], labels))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
