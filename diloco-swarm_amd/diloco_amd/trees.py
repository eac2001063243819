"""Parameter trees the outer step walks: GPT-2 `parameters()` order and shapes.

Restates the order `src/model.py:104-125` (GPT2.__init__) produces: transformer.wte,
transformer.wpe, per block ln_1 / attn.c_attn / attn.c_proj / ln_2 / mlp.c_fc / mlp.c_proj
(weight then bias), ln_f, and lm_head unless tied to wte (`parameter_sharing`,
src/model.py:119-120; `parameters()` yields a shared tensor once, under its first name).
Pinned against the reference import by tests/golden/trees.json.

Named trees:
  micro : GPT2Config(n_layer=2, n_head=2, n_embd=32, vocab_size=96, block_size=16), tied
  tiny  : (4, 4, 128), untied (configs/model/gpt2-tiny.toml; ModelConfig default untied)
  t125  : (12, 12, 768), tied     -> 148 tensors, 124,475,904 params
  t1.3b : (24, 16, 2048), tied    -> 292 tensors, 1,313,722,368 params
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Tuple


@dataclass(frozen=True)
class TreeSpec:
    name: str
    n_layer: int
    n_head: int
    n_embd: int
    vocab_size: int = 50304
    block_size: int = 1024
    tied: bool = True
    bias: bool = True

    def params(self) -> List[Tuple[str, Tuple[int, ...]]]:
        C, V, B = self.n_embd, self.vocab_size, self.block_size
        out: List[Tuple[str, Tuple[int, ...]]] = [
            ("transformer.wte.weight", (V, C)),
            ("transformer.wpe.weight", (B, C)),
        ]
        for i in range(self.n_layer):
            p = f"transformer.h.{i}."
            blk = [
                ("ln_1.weight", (C,)), ("ln_1.bias", (C,)),
                ("attn.c_attn.weight", (3 * C, C)), ("attn.c_attn.bias", (3 * C,)),
                ("attn.c_proj.weight", (C, C)), ("attn.c_proj.bias", (C,)),
                ("ln_2.weight", (C,)), ("ln_2.bias", (C,)),
                ("mlp.c_fc.weight", (4 * C, C)), ("mlp.c_fc.bias", (4 * C,)),
                ("mlp.c_proj.weight", (C, 4 * C)), ("mlp.c_proj.bias", (C,)),
            ]
            out += [(p + n, s) for n, s in blk if self.bias or not n.endswith("bias")]
        out += [("transformer.ln_f.weight", (C,))]
        if self.bias:
            out += [("transformer.ln_f.bias", (C,))]
        if not self.tied:
            out += [("lm_head.weight", (V, C))]
        return out

    def numels(self) -> List[int]:
        return [math.prod(s) for _, s in self.params()]

    def total(self) -> int:
        return sum(self.numels())

    def init_spec(self) -> List[Tuple[float, float]]:
        """(base, scale) per tensor for the synthetic outer init (diloco_amd.synth).

        Mirrors the reference init (src/model.py:121-133): LayerNorm weight 1, biases 0,
        Linear/Embedding weights std 0.02, c_proj weights std 0.02/sqrt(2L); drawn uniform
        with that std (scale = std*sqrt(3)) so every generator is exact integer->float.
        """
        out = []
        for name, _ in self.params():
            if name.endswith("bias"):
                out.append((0.0, 0.0))
            elif ".ln_" in name or name.startswith("transformer.ln_f"):
                out.append((1.0, 0.0))
            elif name.endswith("c_proj.weight"):
                out.append((0.0, 0.02 / math.sqrt(2 * self.n_layer) * math.sqrt(3.0)))
            else:
                out.append((0.0, 0.02 * math.sqrt(3.0)))
        return out


TREES = {
    "micro": TreeSpec("micro", n_layer=2, n_head=2, n_embd=32, vocab_size=96, block_size=16),
    "tiny": TreeSpec("tiny", n_layer=4, n_head=4, n_embd=128, tied=False),
    "t125": TreeSpec("t125", n_layer=12, n_head=12, n_embd=768),
    "t1.3b": TreeSpec("t1.3b", n_layer=24, n_head=16, n_embd=2048),
}


def get_tree(name: str) -> TreeSpec:
    try:
        return TREES[name]
    except KeyError:
        raise KeyError(f"unknown tree {name!r}; known: {sorted(TREES)}") from None
