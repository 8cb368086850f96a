"""Test models and data helpers (reference `tests/unit/simple_model.py`)."""
import torch
import torch.nn as nn

from deepspeedsyclsupport_amd.models.llama import LlamaConfig, LlamaForCausalLM


class SimpleModel(nn.Module):

    def __init__(self, hidden_dim, empty_grad=False, nlayers=1):
        super().__init__()
        self.linears = nn.ModuleList([nn.Linear(hidden_dim, hidden_dim) for _ in range(nlayers)])
        if empty_grad:
            self.unused = nn.Linear(hidden_dim, hidden_dim)
        self.cross_entropy_loss = nn.CrossEntropyLoss()

    def forward(self, x, y):
        for l in self.linears:
            x = l(x)
        return self.cross_entropy_loss(x, y)


def tiny_llama_config(**kw):
    d = dict(vocab_size=128, hidden_size=64, intermediate_size=128, num_hidden_layers=2, num_attention_heads=4,
             max_position_embeddings=64)
    d.update(kw)
    return LlamaConfig(**d)


def tiny_llama(seed=0, **kw):
    torch.manual_seed(seed)
    return LlamaForCausalLM(tiny_llama_config(**kw))


def random_tokens(n, batch, seq, vocab=128, seed=1234):
    g = torch.Generator().manual_seed(seed)
    return [torch.randint(0, vocab, (batch, seq), generator=g) for _ in range(n)]


def base_config(stage=0, lr=1e-2, mb=2, gas=1, clip=1.0, dtype="fp32", **extra):
    c = {
        "train_micro_batch_size_per_gpu": mb,
        "gradient_accumulation_steps": gas,
        "optimizer": {"type": "AdamW", "params": {"lr": lr, "weight_decay": 0.01}},
        "zero_optimization": {"stage": stage},
        "gradient_clipping": clip,
        "steps_per_print": 1000,
    }
    if dtype == "bf16":
        c["bf16"] = {"enabled": True}
    elif dtype == "fp16":
        c["fp16"] = {"enabled": True, "initial_scale_power": 8}
    c.update(extra)
    return c
