"""ViT-B/16 (torchvision ``vit_b_16`` module tree and state_dict names) on ringdp's kernels.

BASELINE.json config 5 ("ViT-B/16 synthetic DDP fp8 on 8xMI355X").  torchvision is not part of this
stack, so the architecture is defined here with the same names: ``conv_proj``, ``class_token``,
``encoder.pos_embedding``, ``encoder.layers.encoder_layer_{i}.{ln_1, self_attention, ln_2, mlp}``,
``encoder.ln``, ``heads.head`` - and the same initialisation.

GPU path (``forward`` on CUDA tensors): token rows are bf16 ``[B*T, 768]``; each encoder block is
LN -> fused QKV GEMM (+bias) -> attention (batched MFMA GEMMs + softmax kernel) -> out-proj GEMM
with the residual add in its epilogue -> LN -> MLP-1 GEMM with bias+GELU epilogue (pre-activation
kept) -> MLP-2 GEMM with the residual add in its epilogue.  CPU path: plain ATen modules.
"""
from __future__ import annotations

import math
from collections import OrderedDict

import torch
import torch.nn as nn

from ..ops.transformer import (AttentionF, ClassRowsF, LayerNormF, LayerNormFork, MLPF, MLPF8, PatchTokensF,
                                cast_weights, clear_weights, fp8_enabled, fp8_mlp_fusable, layernorm_fork, linear)


class MLPBlock(nn.Sequential):
    def __init__(self, dim: int, hidden: int, dropout: float = 0.0):
        super().__init__(nn.Linear(dim, hidden), nn.GELU(), nn.Dropout(dropout), nn.Linear(hidden, dim),
                         nn.Dropout(dropout))
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.xavier_uniform_(m.weight)
                nn.init.normal_(m.bias, std=1e-6)


class EncoderBlock(nn.Module):
    def __init__(self, heads: int, dim: int, mlp_dim: int, dropout: float = 0.0, attention_dropout: float = 0.0):
        super().__init__()
        self.num_heads = heads
        self.ln_1 = nn.LayerNorm(dim, eps=1e-6)
        self.self_attention = nn.MultiheadAttention(dim, heads, dropout=attention_dropout, batch_first=True)
        self.dropout = nn.Dropout(dropout)
        self.ln_2 = nn.LayerNorm(dim, eps=1e-6)
        self.mlp = MLPBlock(dim, mlp_dim, dropout)

    def forward(self, x):  # ATen path, x [B, T, D]
        h = self.ln_1(x)
        h, _ = self.self_attention(h, h, h, need_weights=False)
        x = x + self.dropout(h)
        return x + self.mlp(self.ln_2(x))

    def forward_rows(self, x, B: int, T: int):  # ringdp path, x [B*T, D] bf16
        att = self.self_attention
        if fp8_enabled():  # fp8 linears (LinearF's quantised path); residual gradients join in the LN backward
            fc1, fc2 = self.mlp[0], self.mlp[3]
            h, x = layernorm_fork(x, self.ln_1, att.in_proj_weight)
            qkv = _lin(h, att.in_proj_weight, att.in_proj_bias)
            o = AttentionF.apply(qkv, B, T, self.num_heads)
            x = linear(o, att.out_proj, residual=x)
            h, x = layernorm_fork(x, self.ln_2, fc1.weight)
            if fp8_mlp_fusable(h.shape[0], h.shape[1], fc1.weight.shape[0]):  # e4m3 from the GEMM epilogues
                return MLPF8.apply(h, fc1.weight, fc1.bias, fc2.weight, fc2.bias, x)
            h = linear(h, fc1, act=2)
            return linear(h, fc2, residual=x)
        # bf16: the residual streams' gradients join in the LayerNorm backward kernels (LayerNormFork)
        # and the GELU backward runs in fc2's data-gradient epilogue (MLPF)
        h, x = LayerNormFork.apply(x, self.ln_1.weight, self.ln_1.bias, self.ln_1.eps)
        qkv = _lin(h, att.in_proj_weight, att.in_proj_bias)
        o = AttentionF.apply(qkv, B, T, self.num_heads)
        x = linear(o, att.out_proj, residual=x)
        h, x = LayerNormFork.apply(x, self.ln_2.weight, self.ln_2.bias, self.ln_2.eps)
        fc1, fc2 = self.mlp[0], self.mlp[3]
        return MLPF.apply(h, fc1.weight, fc1.bias, fc2.weight, fc2.bias, x)


def _lin(x, w, b):
    from ..ops.transformer import LinearF

    return LinearF.apply(x, w, b, None, 0, False)


class Encoder(nn.Module):
    def __init__(self, seq_length: int, num_layers: int, heads: int, dim: int, mlp_dim: int, dropout: float = 0.0,
                 attention_dropout: float = 0.0):
        super().__init__()
        self.pos_embedding = nn.Parameter(torch.empty(1, seq_length, dim).normal_(std=0.02))
        self.dropout = nn.Dropout(dropout)
        self.layers = nn.Sequential(OrderedDict(
            (f"encoder_layer_{i}", EncoderBlock(heads, dim, mlp_dim, dropout, attention_dropout))
            for i in range(num_layers)))
        self.ln = nn.LayerNorm(dim, eps=1e-6)

    def forward(self, x):
        return self.ln(self.layers(self.dropout(x + self.pos_embedding)))


class VisionTransformer(nn.Module):
    def __init__(self, image_size: int = 224, patch_size: int = 16, num_layers: int = 12, num_heads: int = 12,
                 hidden_dim: int = 768, mlp_dim: int = 3072, num_classes: int = 1000, dropout: float = 0.0):
        super().__init__()
        self.image_size, self.patch_size, self.hidden_dim = image_size, patch_size, hidden_dim
        self.conv_proj = nn.Conv2d(3, hidden_dim, kernel_size=patch_size, stride=patch_size)
        seq_length = (image_size // patch_size) ** 2 + 1
        self.class_token = nn.Parameter(torch.zeros(1, 1, hidden_dim))
        self.encoder = Encoder(seq_length, num_layers, num_heads, hidden_dim, mlp_dim, dropout)
        self.seq_length = seq_length
        self.heads = nn.Sequential(OrderedDict(head=nn.Linear(hidden_dim, num_classes)))
        fan_in = 3 * patch_size * patch_size
        nn.init.trunc_normal_(self.conv_proj.weight, std=math.sqrt(1 / fan_in))
        nn.init.zeros_(self.conv_proj.bias)
        nn.init.zeros_(self.heads.head.weight)
        nn.init.zeros_(self.heads.head.bias)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.is_cuda:
            return self.forward_rows(x)
        return self.reference_forward(x)

    def reference_forward(self, x: torch.Tensor) -> torch.Tensor:
        n = x.shape[0]
        x = self.conv_proj(x.float()).reshape(n, self.hidden_dim, -1).permute(0, 2, 1)
        x = torch.cat([self.class_token.expand(n, -1, -1), x], dim=1)
        x = self.encoder(x)
        return self.heads(x[:, 0])

    def forward_rows(self, x: torch.Tensor) -> torch.Tensor:
        B, T = x.shape[0], self.seq_length
        # every linear weight's bf16 copy in one launch (instead of one cast per linear)
        ws = []
        for blk in self.encoder.layers:
            att = blk.self_attention
            ws += [att.in_proj_weight, att.out_proj.weight, blk.mlp[0].weight, blk.mlp[3].weight]
        cast_weights(ws)
        try:
            h = PatchTokensF.apply(x, self.conv_proj.weight, self.conv_proj.bias, self.class_token,
                                   self.encoder.pos_embedding, self.patch_size)
            for blk in self.encoder.layers:
                h = blk.forward_rows(h, B, T)
        finally:
            clear_weights()
        ln = self.encoder.ln
        h = LayerNormF.apply(h, ln.weight, ln.bias, ln.eps)
        cls = ClassRowsF.apply(h, B, T)
        return linear(cls, self.heads.head, out_f32=True)


def vit_b_16(num_classes: int = 1000, image_size: int = 224, **kw) -> VisionTransformer:
    return VisionTransformer(image_size=image_size, patch_size=16, num_layers=12, num_heads=12, hidden_dim=768,
                             mlp_dim=3072, num_classes=num_classes, **kw)


def vit_tiny(num_classes: int = 10, image_size: int = 32, **kw) -> VisionTransformer:
    """Small config for tests: 4x4 patches, 4 layers, 64-dim (shapes exercise the same kernels)."""
    return VisionTransformer(image_size=image_size, patch_size=4, num_layers=2, num_heads=4, hidden_dim=64,
                             mlp_dim=128, num_classes=num_classes, **kw)
