"""CPU restatement of the reference's training step — TEST INFRASTRUCTURE ONLY.

Only tests/ import this (the checker for oaz_trainer_*); the product path never does.
It restates, in float64 torch on the CPU (the same ATen ops tch calls):
  ConvResNet::forward(train=true)     alphazero-training/src/net.rs:35-66,101-232
      BN in training mode on batch statistics, running stats updated with momentum 0.1 and
      the unbiased variance (tch nn::batch_norm2d defaults)
  ConvResNet::alphaloss               net.rs:234-243
      value: mean((z - v)^2) with z of shape [B] (Tensor::from(f64) stacks to [B],
      train.rs:64,284-291) against v [B,1]: broadcast to [B,B] (quirk Q16; `broadcast=False`
      gives the elementwise loss)
      policy: -(log(p) * pi).sum(dim 1).mean() over p, pi [B,2,25] (sums the 2 card rows, then
      averages over B*25 entries)
  opt.backward_step                   train.rs:181-186,309
      torch SGD: d = g + wd*p; buf = momentum*buf + d (buf = d at the first step); p -= lr*buf,
      over the trainable variables (conv/linear weights and biases, BN gamma/beta).
Parity is "unpinned" against the reference binary itself (Rust/tch cannot be built here,
SURVEY.md 8c); this follows the op graph of net.rs/train.rs line by line.
"""
from __future__ import annotations

from typing import Dict, Tuple

import numpy as np
import torch
import torch.nn.functional as F

RUNNING = ("running_mean", "running_var")


def _bn(x, named, name, train):
    return F.batch_norm(x, named[f"{name}|running_mean"], named[f"{name}|running_var"], named[f"{name}|weight"],
                        named[f"{name}|bias"], training=train, momentum=0.1, eps=1e-5)


def forward(named: Dict[str, torch.Tensor], x: torch.Tensor, blocks: int, train: bool = True):
    """net.rs: trunk conv_init_1/bn1/relu, `blocks` x ResNetBlock, value and policy heads."""
    y = F.relu(_bn(F.conv2d(x, named["conv_init_1|weight"], named["conv_init_1|bias"], padding=1), named, "bn1",
                   train))
    for i in range(blocks):
        p1 = f"resnet_{i}|resnet_small_block1"
        p2 = f"resnet_{i}|resnet_small_block2"
        h = F.relu(_bn(F.conv2d(y, named[f"{p1}|small_block_conv|weight"], named[f"{p1}|small_block_conv|bias"],
                                padding=1), named, f"{p1}|small_block_bn", train))
        h = _bn(F.conv2d(h, named[f"{p2}|small_block_conv|weight"], named[f"{p2}|small_block_conv|bias"], padding=1),
                named, f"{p2}|small_block_bn", train)
        y = F.relu(h + y)
    v = F.relu(_bn(F.conv2d(y, named["vh_conv|weight"], named["vh_conv|bias"]), named, "vh_bn", train))
    v = F.relu(F.linear(v.flatten(1), named["vh_linear1|weight"], named["vh_linear1|bias"]))
    v = torch.tanh(F.linear(v, named["vh_linear2|weight"], named["vh_linear2|bias"]))
    p = F.relu(_bn(F.conv2d(y, named["policy_conv|weight"], named["policy_conv|bias"]), named, "policy_bn", train))
    p = torch.softmax(F.linear(p.flatten(1), named["ph_linear2|weight"], named["ph_linear2|bias"]), -1)
    return p.reshape(-1, 2, 25), v


def alphaloss(v, p, pi, z, broadcast: bool = True):
    zz = z if broadcast else z.reshape(-1, 1)
    diff = zz - v
    value_loss = (diff * diff).mean()
    policy_loss = -(p.log() * pi).sum(1).mean()
    return value_loss, policy_loss


def train_step(named_np: Dict[str, np.ndarray], planes: np.ndarray, pi: np.ndarray, z: np.ndarray, blocks: int,
               lr: float = 5e-3, momentum: float = 0.9, wd: float = 1e-4, bufs: Dict[str, torch.Tensor] = None,
               broadcast: bool = True) -> Tuple[Dict[str, np.ndarray], Dict[str, np.ndarray], float, float, dict]:
    """One step; returns (new named params incl. running stats, grads, value loss, policy loss,
    momentum buffers)."""
    named = {k: torch.tensor(np.asarray(v, dtype=np.float64), requires_grad=not k.endswith(RUNNING))
             for k, v in named_np.items()}
    with torch.no_grad():
        for k, t in named.items():
            if k.endswith(RUNNING):
                t.requires_grad_(False)
    x = torch.tensor(np.asarray(planes, dtype=np.float64))
    p, v = forward(named, x, blocks, train=True)
    lv, lp = alphaloss(v, p, torch.tensor(np.asarray(pi, dtype=np.float64)).reshape(-1, 2, 25),
                       torch.tensor(np.asarray(z, dtype=np.float64)), broadcast)
    (lv + lp).backward()
    bufs = {} if bufs is None else bufs
    grads, out = {}, {}
    with torch.no_grad():
        for k, t in named.items():
            if k.endswith(RUNNING):
                out[k] = t.numpy().copy()
                continue
            g = t.grad.clone()
            grads[k] = g.numpy().copy()
            d = g + wd * t
            if k in bufs:
                bufs[k] = momentum * bufs[k] + d
            else:
                bufs[k] = d.clone()
            out[k] = (t - lr * bufs[k]).numpy().copy()
    return out, grads, float(lv.detach()), float(lp.detach()), bufs
