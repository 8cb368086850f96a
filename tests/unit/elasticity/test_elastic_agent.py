"""Failure detection + elastic restart + checkpoint resume, end to end on CPU/gloo (reference
`elasticity/elastic_agent.py` DSElasticAgent; SURVEY §5.3 fault-injection design item).

A 2-rank ZeRO-2 job checkpoints every step; rank 1 is made to crash (or hang) at step 3 of attempt 0. The agent must
detect it, restart the group, and the restarted ranks must resume from the last checkpoint and finish with the
same weights as an uninterrupted run."""
import json
import os
import subprocess
import sys
import textwrap

import pytest
import torch

from deepspeedsyclsupport_amd.elasticity.elastic_agent import DSElasticAgent, WorkerSpec

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

SCRIPT = textwrap.dedent("""
    import json, os, sys, torch
    sys.path.insert(0, {repo!r})
    sys.path.insert(0, {tests!r})
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    from unit.simple_model import base_config, random_tokens, tiny_llama
    ds.init_distributed(dist_backend="gloo")
    cfg = base_config(stage=2, lr=1e-2, mb=2, clip=1.0)
    eng, _, _, _ = ds.initialize(model=tiny_llama(), config=cfg)
    ck = {ckpt!r}
    start = 0
    if os.path.exists(os.path.join(ck, "latest")):
        _, client = eng.load_checkpoint(ck)
        start = client["next_step"]
    data = random_tokens(6, 2, 16, seed=7 + dist.get_rank())
    for i in range(start, 6):
        loss = eng(data[i], labels=data[i])
        eng.backward(loss)
        eng.step()
        eng.save_checkpoint(ck, tag=f"s{{i}}", client_state={{"next_step": i + 1}})
    if dist.get_rank() == 0:
        torch.save({{n: p.detach().float().clone() for n, p in eng.module.named_parameters()}}, {out!r})
        with open({out!r} + ".json", "w") as f:
            json.dump({{"attempt": int(os.environ.get("TORCHELASTIC_RESTART_COUNT", 0)), "start": start}}, f)
""")


def _run(tmp, tag, fault, timeout_hb=0.0, restarts=2):
    ck, out = str(tmp / f"ck_{tag}"), str(tmp / f"w_{tag}.pt")
    script = tmp / f"train_{tag}.py"
    script.write_text(SCRIPT.format(repo=REPO, tests=os.path.join(REPO, "tests"), ckpt=ck, out=out))
    env = {"DS_FAULT_INJECT": fault} if fault else {}
    hb = str(tmp / f"hb_{tag}") if timeout_hb else None
    if hb:
        os.makedirs(hb, exist_ok=True)
    spec = WorkerSpec(cmd=[sys.executable, str(script)], nproc=2, env=env, max_restarts=restarts,
                      log_dir=str(tmp / f"logs_{tag}"), heartbeat_dir=hb, heartbeat_timeout=timeout_hb)
    res = DSElasticAgent(spec).run()
    return res, out


@pytest.mark.parametrize("mode", ["exit", "raise", "hang"])
def test_restart_and_resume(tmp_path, mode):
    ref, ref_out = _run(tmp_path, "ref", None)
    assert ref.state == "SUCCEEDED" and ref.restarts == 0
    hb = 20.0 if mode == "hang" else 0.0
    got, got_out = _run(tmp_path, mode, f"rank=1,step=3,mode={mode}", timeout_hb=hb)
    assert got.state == "SUCCEEDED" and got.restarts == 1, got
    meta = json.load(open(got_out + ".json"))
    # the fault fires inside step 3 (before its checkpoint): the second attempt resumes from the step-2 checkpoint
    assert meta == {"attempt": 1, "start": 2}
    w_ref = torch.load(ref_out, weights_only=True)
    w_got = torch.load(got_out, weights_only=True)
    for n in w_ref:
        torch.testing.assert_close(w_got[n], w_ref[n], rtol=0, atol=0, msg=n)


def test_gives_up_after_max_restarts(tmp_path):
    res, _ = _run(tmp_path, "dead", "rank=0,step=1,mode=exit;rank=0,step=1,mode=exit,attempt=1", restarts=1)
    assert res.state == "FAILED" and res.restarts == 1
