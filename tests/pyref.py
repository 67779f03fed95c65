"""Second, independent restatement of the reference search in pure Python — TEST INFRASTRUCTURE.

Written directly from the Rust (rules: onitama-game/src/game/state.rs, card.rs; search:
alphazero-training/src/alphazero_mcts/mcts_arena.rs) without looking at the C oracle, and used
only to cross-check the oracle's MCTS on small cases (noise off, HASH evaluator). Slow: keep
sims and positions small.
"""
from __future__ import annotations

import math
import struct
from dataclasses import dataclass, field
from typing import List, Optional

M64 = (1 << 64) - 1
CARD_POS = [0x20004000, 0x0440A000, 0x02202000, 0x00828000, 0x01220000, 0x02940000, 0x02142000,
            0x00948000, 0x0280A000, 0x02804000, 0x0100A000, 0x01104000, 0x01044000, 0x01140000,
            0x02048000, 0x00902000]
CARD_MIR = [0x01000200, 0x02811000, 0x02022000, 0x00A08000, 0x00224000, 0x0014A000, 0x02142000,
            0x00948000, 0x0280A000, 0x0100A000, 0x02804000, 0x01044000, 0x01104000, 0x00144000,
            0x00902000, 0x02048000]
FILE_A, FILE_E, FILE_AB, FILE_DE = 0x84210800, 0x08421080, 0xC6318C00, 0x18C63180
U32 = 0xFFFFFFFF


def _maps_for(card):  # card.rs:553-604
    m = [0] * 25
    m[12] = card
    for n in range(1, 13):
        left = (card << n) & 0xFFFFFF80 & U32
        right = (card >> n) & 0xFFFFFF80
        r = n % 5
        if r == 1:
            left &= ~FILE_E & U32; right &= ~FILE_A & U32
        elif r == 2:
            left &= ~FILE_DE & U32; right &= ~FILE_AB & U32
        elif r == 3:
            left &= ~FILE_AB & U32; right &= ~FILE_DE & U32
        elif r == 4:
            left &= ~FILE_A & U32; right &= ~FILE_E & U32
        m[12 - n], m[12 + n] = left, right
    return m


ATTACK = [[_maps_for(CARD_MIR[c] if p else CARD_POS[c]) for c in range(16)] for p in range(2)]


def bit(x, n):
    return (x >> (31 - n)) & 1


@dataclass
class S:
    kings: List[int]
    pawns: List[int]
    cards: List[int]
    color: int

    def copy(self):
        return S(list(self.kings), list(self.pawns), list(self.cards), self.color)


def legal_moves(s: S, color: int):  # state.rs:301-378
    out = []
    for slot in ((0, 1) if color == 0 else (2, 3)):
        pawns, king = s.pawns[color], s.kings[color]
        for n in range(25):
            pb, kb = bit(pawns, n), bit(king, n)
            if not pb and not kb:
                continue
            am = ATTACK[color][s.cards[slot]][n]
            if pb:
                mp, piece = ((am | pawns) & ~pawns) & ~king & U32, 0
            else:
                mp, piece = ((am | king) & ~king) & ~pawns & U32, 1
            for i in range(25):
                if bit(mp, i):
                    out.append((slot, n, i, piece))
    return out


def make_move(s: S, mv, color):  # state.rs:145-202 -> 0 Capture 1 RedWin 2 BlueWin 3 InProgress
    slot, fr, to, piece = mv
    res = 3
    if piece == 0:
        s.pawns[color] &= ~(1 << (31 - fr)) & U32
    else:
        s.kings[color] &= ~(1 << (31 - fr)) & U32
    e = color ^ 1
    if bit(s.pawns[e], to):
        s.pawns[e] &= ~(1 << (31 - to)) & U32
        res = 0
    elif bit(s.kings[e], to):
        s.kings[e] &= ~(1 << (31 - to)) & U32
        res = 1 if color == 0 else 2
    if piece == 0:
        s.pawns[color] |= 1 << (31 - to)
    else:
        s.kings[color] |= 1 << (31 - to)
    if piece == 1 and ((color == 0 and to == 2) or (color == 1 and to == 22)):
        res = 1 if color == 0 else 2
    s.cards[slot], s.cards[4] = s.cards[4], s.cards[slot]
    return res


def current_state(s: S):  # state.rs:120-134
    if s.kings[0] == 0 or s.kings[1] == 0x200:
        return 2
    if s.kings[1] == 0 or s.kings[0] == 0x20000000:
        return 1
    return 3


def _sm(x):
    z = (x + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def _f32(x):
    return struct.unpack("f", struct.pack("f", x))[0]


def hash_eval(s: S):  # the HASH test evaluator, fp32-exact values
    h = _sm(s.kings[0] | (s.kings[1] << 32))
    h = _sm(h ^ (s.pawns[0] | (s.pawns[1] << 32)))
    c = (s.cards[0] | s.cards[1] << 4 | s.cards[2] << 8 | s.cards[3] << 12 | s.cards[4] << 16 | s.color << 20)
    h = _sm(h ^ c)
    pol = [_f32(((_sm((h + i) & M64) >> 40) + 1) / 16777216.0) for i in range(50)]
    v = _f32(((_sm(h ^ 0x5DEECE66D) >> 40) - 8388608) / 8388608.0)
    return pol, v


@dataclass
class Node:  # mcts_arena.rs:355-373
    parent: Optional[int]
    mov: Optional[tuple]
    color: int
    prob: float
    children: List[int] = field(default_factory=list)
    visits: int = 0
    reward: float = 0.0
    winrate: float = 0.0
    terminal: bool = False
    expanded: bool = False


def _key(x):  # f64::total_cmp
    i = struct.unpack("<q", struct.pack("<d", x))[0]
    return i ^ ((i >> 63) & 0x7FFFFFFFFFFFFFFF)


def search(root: S, sims: int, c: float, evaluator=hash_eval):
    """Noise-free AlphaZero search (mcts_arena.rs:75-124). Returns (move, pi[50], arena)."""
    arena = [Node(None, None, root.color, 1.0)]

    def reward(res, color):
        if res == 1:
            return 1.0 if color == 0 else -1.0
        if res == 2:
            return 1.0 if color == 1 else -1.0
        return 0.0

    for _ in range(sims):
        gs = root.copy()
        node = 0
        while arena[node].expanded and not arena[node].terminal:
            if not arena[node].children:  # defined behaviour for the reference panic (Q6)
                break
            p = arena[node]
            best, bk = None, None
            for ci in p.children:
                ch = arena[ci]
                u = ch.winrate + c * ch.prob * (math.sqrt(float(p.visits)) / float(ch.visits + 1))
                k = _key(u)
                if best is None or not (bk > k):
                    best, bk = ci, k
            node = best
            res = make_move(gs, arena[node].mov, arena[arena[node].parent].color)
            gs.color ^= 1
            if res in (1, 2):
                arena[node].terminal = True
        pol, val = evaluator(gs)
        moves = legal_moves(gs, gs.color)
        pri = [[0.0] * 25, [0.0] * 25]
        for (slot, fr, to, piece) in moves:
            pri[slot % 2][to] = float(pol[(slot % 2) * 25 + to])
        for r in range(2):
            tot = 0.0
            for x in pri[r]:
                tot += x
            if tot > 0.0:
                pri[r] = [x / tot for x in pri[r]]
        if not arena[node].expanded and not arena[node].terminal:
            for mv in moves:
                arena.append(Node(node, mv, arena[node].color ^ 1, pri[mv[0] % 2][mv[2]]))
                arena[node].children.append(len(arena) - 1)
            arena[node].expanded = True
        parent = arena[node].parent if arena[node].parent is not None else 0
        rc = arena[parent].color
        mr = current_state(gs)
        r = reward(mr, rc) if mr in (1, 2) else float(val)
        idx = node
        while True:
            nd = arena[idx]
            nd.visits += 1
            nd.reward += r
            nd.winrate = nd.reward / nd.visits
            if nd.parent is None:
                break
            idx = nd.parent
            r = -r
    rootn = arena[0]
    pi = [0.0] * 50
    for ci in rootn.children:
        ch = arena[ci]
        pi[(ch.mov[0] % 2) * 25 + ch.mov[2]] += ch.visits
    tot = _f32(sum(pi))
    pi = [_f32(_f32(x) / tot) if tot > 0 else 0.0 for x in pi]
    best = None
    for ci in rootn.children:
        if best is None or not (arena[best].visits / rootn.visits > arena[ci].visits / rootn.visits):
            best = ci
    return (arena[best].mov if best is not None else None), pi, arena
