"""Stream-concurrency micro test of two independent block-step chains."""
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import svdj  # noqa: E402

K = svdj.ops.kernels
dev = torch.device("cuda:0")
n, W = 4096, 32
A = torch.rand(n, n, device=dev)
pairs = torch.from_numpy(svdj.parallel.schedule.round_robin(n // W // 2)).to(dev)
A1, A2 = A[: n // 2].clone(), A[n // 2:].clone()


def state(X):
    Vt = torch.zeros(X.shape[0], 4096, device=dev)
    K.set_identity(Vt, X.shape[0])
    return Vt, K.col_norms2(X, n), K.new_metric(dev)


st = [state(A1), state(A2)]
s = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
modes = [0] * pairs.shape[0]


def launch(i, X):
    Vt, D, m = st[i]
    K.block_steps(X, Vt, D, n, pairs, W, modes, 1e-30, 1, m, i)


def run(mode):
    torch.cuda.synchronize()
    t = time.perf_counter()
    if mode == "seq":
        launch(0, A1)
        launch(1, A2)
    elif mode == "plain":
        for i, X in enumerate((A1, A2)):
            with torch.cuda.stream(s[i]):
                launch(i, X)
    elif mode in ("event_null", "event_side"):
        main = torch.cuda.current_stream(dev)
        ready = torch.cuda.Event()
        ready.record(main)
        for i, X in enumerate((A1, A2)):
            s[i].wait_event(ready)
            with torch.cuda.stream(s[i]):
                launch(i, X)
        for x in s:
            main.wait_stream(x)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) * 1e3


side_main = torch.cuda.Stream(dev)
for mode in ["seq", "plain", "event_null", "seq", "plain", "event_null"]:
    print(mode, "%.2f ms" % run(mode), flush=True)
with torch.cuda.stream(side_main):
    for _ in range(2):
        print("event_side(main=non-default)", "%.2f ms" % run("event_side"), flush=True)
