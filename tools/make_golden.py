"""Generate the NN golden fixtures under tests/golden/ (run in the build container, where the
reference is mounted; the GPU box only reads the committed outputs).

  weights_3block_trained.npy   the reference's trained 3-block net (models/model_5e-3_3_resnet.ot)
                               as a canonical fp32 blob, read with the no-unpickling .ot reader
  weights_5block_trained.npy   the reference's trained 5-block net (models/model_5e-3.ot), likewise
  nn_golden.npz                seeded positions (random play driven by the C oracle's rules) and
                               torch-CPU outputs of the net.rs op graph (F.conv2d, F.batch_norm
                               eval eps=1e-5, relu, linear, tanh, softmax) for:
                                 trained3  - the trained 3-block weights
                                 random3   - engine random init, seed 0, 3 blocks
                                 random6   - engine random init, seed 1, 6 blocks
NOTE: torch 2.10 CPU arithmetic stands in for the reference's libtorch 1.13.1 (tch 0.10.3);
both are fp32 ATen CPU kernels, so parity is "within 1e-4", never bitwise.
Run: python tools/make_golden.py
"""
import random
import sys
from pathlib import Path

import numpy as np
import torch
import torch.nn.functional as F

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT / "onitama-alphazero_amd"))

import oracle_ffi as orc  # noqa: E402
from onitama_az import _abi  # noqa: E402
from onitama_az.weights import (blob_from_named, named_from_blob, random_weights,  # noqa: E402
                                read_ot)

GOLD = ROOT / "tests" / "golden"
REF_MODEL = Path("/root/reference/models/model_5e-3_3_resnet.ot")
REF_MODEL5 = Path("/root/reference/models/model_5e-3.ot")


def random_positions(n: int, seed: int) -> np.ndarray:
    """Positions from seeded random play (rules = C oracle), both colours, all game phases."""
    rng = random.Random(seed)
    out = []
    game = 0
    while len(out) < n:
        deck = orc.deal_deck(seed, game)
        game += 1
        s = orc.initial_state(deck)
        plies = rng.randint(0, 40)
        for _ in range(plies):
            moves = orc.movegen(s)
            if len(moves) == 0:
                break
            m = moves[rng.randrange(len(moves))]
            color = int(s["to_move"][0])
            r = orc.make_move(s, tuple(int(m[k]) for k in ("from_", "to", "piece", "slot")), color)
            s["to_move"][0] ^= 1
            if r in (1, 2):
                break
        out.append(s.copy())
    return np.concatenate(out)


def torch_forward(named, blocks, planes):
    t = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in named.items()}
    x = torch.from_numpy(planes)

    def cbn(x, conv, bn, pad):
        y = F.conv2d(x, t[f"{conv}|weight"], t[f"{conv}|bias"], stride=1, padding=pad)
        return F.batch_norm(y, t[f"{bn}|running_mean"], t[f"{bn}|running_var"], t[f"{bn}|weight"],
                            t[f"{bn}|bias"], training=False, eps=1e-5)

    with torch.no_grad():
        y = F.relu(cbn(x, "conv_init_1", "bn1", 1))
        for i in range(blocks):
            p = f"resnet_{i}|resnet_small_block"
            y1 = F.relu(cbn(y, f"{p}1|small_block_conv", f"{p}1|small_block_bn", 1))
            y2 = cbn(y1, f"{p}2|small_block_conv", f"{p}2|small_block_bn", 1)
            y = F.relu(y2 + y)
        v = F.relu(cbn(y, "vh_conv", "vh_bn", 0)).flatten(1)
        v = F.relu(F.linear(v, t["vh_linear1|weight"], t["vh_linear1|bias"]))
        v = torch.tanh(F.linear(v, t["vh_linear2|weight"], t["vh_linear2|bias"]))
        p = F.relu(cbn(y, "policy_conv", "policy_bn", 0)).flatten(1)
        p = F.softmax(F.linear(p, t["ph_linear2|weight"], t["ph_linear2|bias"]), dim=-1).reshape(-1, 2, 25)
    return p.numpy(), v.numpy().reshape(-1)


def main():
    torch.set_num_threads(4)
    GOLD.mkdir(parents=True, exist_ok=True)
    trained = read_ot(str(REF_MODEL))
    w3 = blob_from_named(trained, 3)
    np.save(GOLD / "weights_3block_trained.npy", w3)
    np.save(GOLD / "weights_5block_trained.npy", blob_from_named(read_ot(str(REF_MODEL5)), 5))
    states = random_positions(256, seed=7)
    planes = np.stack([orc.encode(s) for s in states])
    out = {"states": states}
    for name, blob, blocks in (("trained3", w3, 3), ("random3", random_weights(0, 3), 3),
                               ("random6", random_weights(1, 6), 6)):
        p, v = torch_forward(named_from_blob(blob, blocks), blocks, planes)
        out[f"policy_{name}"] = p.astype(np.float32)
        out[f"value_{name}"] = v.astype(np.float32)
    np.savez_compressed(GOLD / "nn_golden.npz", **out)
    print("wrote", GOLD / "nn_golden.npz", {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
