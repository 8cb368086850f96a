#!/usr/bin/env python3
"""Does splitting the widest GEMMs of the Llama-2-7B step (gate_up: 22016 features, T = 32768 tokens) into two
library calls run faster than one call? Forward, weight-gradient (K-major operands) and data-gradient products, each
formulation tuned by TunableOp; one JSON line per product."""
import json
import os
import threading
import time

import torch

T, I2, H = 32768, 22016, 4096
I = I2 // 2


def timed(fn, iters=10):
    fn()
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_max_tuning_duration(20)
    tun.set_max_tuning_iterations(10)
    tun.set_filename(os.path.join("gpurun_out", "probe_gemm_split_tunable.csv"), False)
    t0 = time.time()

    def hb():
        while True:
            time.sleep(20)
            print(f"# alive {time.time() - t0:.0f}s", flush=True)

    threading.Thread(target=hb, daemon=True).start()
    bf = dict(device="cuda", dtype=torch.bfloat16)
    fl = 2.0 * T * I2 * H

    def emit(name, res):
        print(json.dumps({"product": name, **{k: f"{v:.3f} ms {fl / v / 1e12:.2f} PF/s" for k, v in res.items()}}),
              flush=True)

    # forward y[T, 2I] = x[T, H] . W[2I, H]^T
    x = torch.randn(T, H, **bf)
    W = torch.randn(I2, H, **bf) * 0.02
    y = torch.empty(T, I2, **bf)
    res = {"one_call": timed(lambda: torch.mm(x, W.t(), out=y))}

    def split_n():
        torch.mm(x, W[:I].t(), out=y[:, :I])
        torch.mm(x, W[I:].t(), out=y[:, I:])

    def split_t(parts):
        def run():
            step = T // parts
            for i in range(parts):
                torch.mm(x[i * step:(i + 1) * step], W.t(), out=y[i * step:(i + 1) * step])
        return run

    res["split_features_2"] = timed(split_n)
    res["split_tokens_2"] = timed(split_t(2))
    res["split_tokens_4"] = timed(split_t(4))
    emit("gate_up forward", res)
    del y

    # weight gradient dW[2I, H] = dyT[2I, T] . xT[H, T]^T
    dyT = torch.randn(I2, T, **bf)
    xT = torch.randn(H, T, **bf)
    dW = torch.empty(I2, H, **bf)
    res = {"one_call": timed(lambda: torch.mm(dyT, xT.t(), out=dW))}

    def wsplit():
        torch.mm(dyT[:I], xT.t(), out=dW[:I])
        torch.mm(dyT[I:], xT.t(), out=dW[I:])

    res["split_features_2"] = timed(wsplit)
    # swap the roles: dW^T[H, 2I] = xT . dyT^T (the down projection's shape class) then no transpose is needed if the
    # caller accepts dW^T -- timing only
    dWt = torch.empty(H, I2, **bf)
    res["transposed_out"] = timed(lambda: torch.mm(xT, dyT.t(), out=dWt))
    emit("gate_up wgrad", res)
    del dyT, xT, dW, dWt

    # data gradient dx[T, H] = dy[T, 2I] . Wt[H, 2I]^T
    dy = torch.randn(T, I2, **bf)
    Wt = torch.randn(H, I2, **bf) * 0.02
    dx = torch.empty(T, H, **bf)
    res = {"one_call": timed(lambda: torch.mm(dy, Wt.t(), out=dx))}

    def dsplit_k():
        torch.mm(dy[:, :I], Wt[:, :I].t(), out=dx)
        dx.addmm_(dy[:, I:], Wt[:, I:].t())

    def dsplit_t(parts):
        def run():
            step = T // parts
            for i in range(parts):
                torch.mm(dy[i * step:(i + 1) * step], Wt.t(), out=dx[i * step:(i + 1) * step])
        return run

    res["split_k_2_accumulate"] = timed(dsplit_k)
    res["split_tokens_2"] = timed(dsplit_t(2))
    res["split_tokens_4"] = timed(dsplit_t(4))
    emit("gate_up dgrad", res)
    del dy, Wt, dx

    # the other forward GEMMs, token split only (a smaller working set per call)
    for name, (n, k) in {"qkv": (12288, 4096), "down": (4096, 11008), "o": (4096, 4096)}.items():
        x = torch.randn(T, k, **bf)
        W = torch.randn(n, k, **bf) * 0.02
        y = torch.empty(T, n, **bf)
        fl = 2.0 * T * n * k
        res = {"one_call": timed(lambda: torch.mm(x, W.t(), out=y))}

        def st():
            torch.mm(x[:T // 2], W.t(), out=y[:T // 2])
            torch.mm(x[T // 2:], W.t(), out=y[T // 2:])

        res["split_tokens_2"] = timed(st)
        emit(name + " forward", res)
        del x, W, y


if __name__ == "__main__":
    main()
