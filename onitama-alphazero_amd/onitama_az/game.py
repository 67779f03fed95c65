"""Python mirror of the reference's game API (onitama-game/src/game/*), backed by the GPU.

Names, argument meaning and error behaviour follow the Rust types so callers (and the tests)
read like the reference's own: State::generate_legal_moves, State::make_move, Deck::rotate,
GameState::progress ... Rule evaluation itself runs in the HIP kernels behind the C ABI
(oaz_movegen / oaz_step / oaz_current_state); there is no Python or CPU implementation of
the rules in the product path.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from enum import IntEnum
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _abi


class PlayerColor(IntEnum):  # player_color.rs:7-10
    Red = 0
    Blue = 1

    def enemy(self) -> "PlayerColor":
        return PlayerColor(self ^ 1)


class PieceKind(IntEnum):  # piece.rs:5-9
    Pawn = 0
    King = 1


class MoveResult(IntEnum):  # move_result.rs:4-9
    Capture = 0
    RedWin = 1
    BlueWin = 2
    InProgress = 3

    def is_win(self) -> bool:  # move_result.rs:11-16
        return self in (MoveResult.RedWin, MoveResult.BlueWin)


@dataclass(frozen=True)
class Card:  # card.rs:5-15
    positions: int
    mirror: int
    player_color: PlayerColor
    index: int


# card.rs:17-463 (positions, mirror, player_color, index)
TIGER = Card(0x2000_4000, 0x0100_0200, PlayerColor.Blue, 0)
DRAGON = Card(0x0440_A000, 0x0281_1000, PlayerColor.Red, 1)
FROG = Card(0x0220_2000, 0x0202_2000, PlayerColor.Red, 2)
RABBIT = Card(0x0082_8000, 0x00A0_8000, PlayerColor.Red, 3)
CRAB = Card(0x0122_0000, 0x0022_4000, PlayerColor.Blue, 4)
ELEPHANT = Card(0x0294_0000, 0x0014_A000, PlayerColor.Red, 5)
GOOSE = Card(0x0214_2000, 0x0214_2000, PlayerColor.Blue, 6)
ROOSTER = Card(0x0094_8000, 0x0094_8000, PlayerColor.Red, 7)
MONKEY = Card(0x0280_A000, 0x0280_A000, PlayerColor.Blue, 8)
MANTIS = Card(0x0280_4000, 0x0100_A000, PlayerColor.Red, 9)
CRANE = Card(MANTIS.mirror, MANTIS.positions, PlayerColor.Blue, 10)
HORSE = Card(0x0110_4000, 0x0104_4000, PlayerColor.Red, 11)
OX = Card(HORSE.mirror, HORSE.positions, PlayerColor.Blue, 12)
BOAR = Card(0x0114_0000, 0x0014_4000, PlayerColor.Red, 13)
EEL = Card(0x0204_8000, 0x0090_2000, PlayerColor.Blue, 14)
COBRA = Card(EEL.mirror, EEL.positions, PlayerColor.Red, 15)

ORIGINAL_CARDS = [TIGER, DRAGON, FROG, RABBIT, CRAB, ELEPHANT, GOOSE, ROOSTER, MONKEY, MANTIS,
                  CRANE, HORSE, OX, BOAR, EEL, COBRA]  # card.rs:465-468
CARD_NAMES = ["Tiger", "Dragon", "Frog", "Rabbit", "Crab", "Elephant", "Goose", "Rooster",
              "Monkey", "Mantis", "Crane", "Horse", "Ox", "Boar", "Eel", "Cobra"]  # card.rs:471-474

RED_CARD1, RED_CARD2, BLUE_CARD1, BLUE_CARD2, NEUTRAL = 0, 1, 2, 3, 4  # deck.rs:14-18

RED_KING_SP = 0x0000_0200  # state.rs:24
BLUE_KING_SP = 0x2000_0000  # state.rs:31
BLUE_PAWNS_SP = 0xD800_0000  # state.rs:38
RED_PAWNS_SP = 0x0000_0D80  # state.rs:45
BLUE_TEMPLE, RED_TEMPLE = 2, 22  # state.rs:48-49


def get_bit(x: int, n: int) -> int:  # common/mod.rs:2-4
    return (x >> (31 - n)) & 1


def from_2d_to_bitboard(value: Tuple[int, int]) -> int:  # common/mod.rs:10-16
    y, x = value
    return 0x8000_0000 >> (y * 5 + x)


def from_2d_to_1d(value: Tuple[int, int]) -> int:  # common/mod.rs:22-25
    y, x = value
    return y * 5 + x


@dataclass(frozen=True, order=True)
class Move:  # move.rs:20-25 (field order = derive(Ord) order)
    from_: int
    to: int
    piece: PieceKind

    @staticmethod
    def from_2d(mov: Tuple[Tuple[int, int], Tuple[int, int]], piece: PieceKind) -> "Move":  # move.rs:107-122
        return Move(from_2d_to_1d(mov[0]), from_2d_to_1d(mov[1]), PieceKind(piece))

    @staticmethod
    def convert_idx_to_notation(idx: int) -> str:  # move.rs:36-48
        return "abcde"[idx % 5] + str(5 - idx // 5)

    @staticmethod
    def convert_notation_to_idx(notation: str) -> int:  # move.rs:51-56
        col = "abcde".index(notation[0])
        row = 5 - int(notation[1])
        if not 0 <= row <= 4:
            raise ValueError("A second character must be in range 1..5!")
        return row * 5 + col


@dataclass(frozen=True)
class DoneMove:  # done_move.rs:3-7
    mov: Move
    used_card_idx: int

    def to_c(self) -> _abi.oaz_move:
        return _abi.oaz_move(self.mov.from_, self.mov.to, int(self.mov.piece), self.used_card_idx)

    @staticmethod
    def from_c(m) -> "DoneMove":
        if isinstance(m, np.void):
            f, t, p, s = (int(m[k]) for k in ("from_", "to", "piece", "slot"))
        else:
            f, t, p, s = m.from_, m.to, m.piece, m.slot
        return DoneMove(Move(f, t, PieceKind(p & 1)), s)

    def is_pass(self) -> bool:
        return self.mov.from_ >= 25


class Deck:  # deck.rs:20-165
    def __init__(self, cards: Sequence[Card]):
        assert len(cards) == 5, "Deck must have 5 random cards"
        self.cards: List[Card] = list(cards)

    @staticmethod
    def default(seed: int = 20260101, game_id: int = 0) -> "Deck":
        """deck.rs:139-151 with the engine's counter-based deal (the reference uses thread_rng)."""
        out = (C.c_uint8 * 5)()
        _abi.load().oaz_deal_deck(C.c_uint64(seed), C.c_uint64(game_id), out)
        return Deck([ORIGINAL_CARDS[i] for i in out])

    def get_player_cards(self, color: PlayerColor) -> List[Card]:  # deck.rs:40-46
        return [self.cards[i] for i in self.get_player_cards_idx(color)]

    @staticmethod
    def get_player_cards_idx(color: PlayerColor) -> List[int]:  # deck.rs:48-53
        return [RED_CARD1, RED_CARD2] if color == PlayerColor.Red else [BLUE_CARD1, BLUE_CARD2]

    def neutral_card(self) -> Card:  # deck.rs:56-58
        return self.cards[NEUTRAL]

    def get_card(self, card_idx: int) -> Card:  # deck.rs:66-69
        assert card_idx < 5
        return self.cards[card_idx]

    def get_card_idx(self, card: Card) -> Optional[int]:
        return self.cards.index(card) if card in self.cards else None

    def rotate(self, idx: int) -> None:  # deck.rs:87-90
        assert idx < 4
        self.cards[idx], self.cards[NEUTRAL] = self.cards[NEUTRAL], self.cards[idx]

    def indices(self) -> List[int]:
        return [c.index for c in self.cards]

    def clone(self) -> "Deck":
        return Deck(self.cards)


class State:  # state.rs:51-56
    def __init__(self, deck: Deck, kings=(RED_KING_SP, BLUE_KING_SP), pawns=(RED_PAWNS_SP, BLUE_PAWNS_SP)):
        self.deck = deck
        self.kings = list(kings)
        self.pawns = list(pawns)

    @staticmethod
    def new(seed: int = 20260101, game_id: int = 0) -> "State":  # state.rs:58-64
        return State(Deck.default(seed, game_id))

    @staticmethod
    def with_deck(deck: Deck) -> "State":  # state.rs:66-72
        return State(deck)

    def clone(self) -> "State":
        return State(self.deck.clone(), self.kings, self.pawns)

    # -- marshalling --
    def to_c(self, color: PlayerColor) -> _abi.oaz_state:
        s = _abi.oaz_state()
        s.kings[0], s.kings[1] = self.kings
        s.pawns[0], s.pawns[1] = self.pawns
        for i, c in enumerate(self.deck.cards):
            s.cards[i] = c.index
        s.to_move = int(color)
        return s

    def to_np(self, color: PlayerColor) -> np.ndarray:
        a = np.zeros(1, dtype=_abi.STATE_DTYPE)
        a["kings"][0] = self.kings
        a["pawns"][0] = self.pawns
        a["cards"][0] = self.deck.indices()
        a["to_move"][0] = int(color)
        return a

    @staticmethod
    def from_np(a) -> Tuple["State", PlayerColor]:
        st = State(Deck([ORIGINAL_CARDS[int(i)] for i in a["cards"]]), [int(x) for x in a["kings"]],
                   [int(x) for x in a["pawns"]])
        return st, PlayerColor(int(a["to_move"]))

    # -- rules (GPU) --
    def is_terminal(self) -> bool:  # state.rs:111-117
        return (self.kings[0] == 0 or self.kings[1] == 0 or self.kings[0] == BLUE_KING_SP
                or self.kings[1] == RED_KING_SP)

    def current_state(self) -> MoveResult:  # state.rs:120-134 (evaluated by the GPU kernel)
        res = np.zeros(1, dtype=np.uint8)
        _abi.check(_abi.load().oaz_current_state(_abi.ptr(self.to_np(PlayerColor.Red)), 1, _abi.ptr(res)))
        return MoveResult(int(res[0]))

    def pass_turn(self, card_idx: int) -> MoveResult:  # state.rs:139-142 `pass`
        self.deck.rotate(card_idx)
        return MoveResult.InProgress

    def make_move(self, mov: Move, player_color: PlayerColor, used_card_idx: int) -> MoveResult:
        """state.rs:145-202 — executed by the GPU step kernel."""
        a = self.to_np(player_color)
        m = np.zeros(1, dtype=_abi.MOVE_DTYPE)
        m[0] = (mov.from_, mov.to, int(mov.piece), used_card_idx)
        res = np.zeros(1, dtype=np.uint8)
        _abi.check(_abi.load().oaz_step(_abi.ptr(a), _abi.ptr(m), 1, _abi.ptr(res)))
        self.kings = [int(x) for x in a["kings"][0]]
        self.pawns = [int(x) for x in a["pawns"][0]]
        self.deck = Deck([ORIGINAL_CARDS[int(i)] for i in a["cards"][0]])
        return MoveResult(int(res[0]))

    def generate_all_legal_moves(self, player_color: PlayerColor) -> List[Tuple[int, Move]]:
        """state.rs:301-310 — (slot, Move) in the reference order, from the GPU movegen kernel."""
        moves, n = movegen_batch(self.to_np(player_color))
        return [(int(m["slot"]), Move(int(m["from_"]), int(m["to"]), PieceKind(int(m["piece"]))))
                for m in moves[0, : n[0]]]

    def generate_legal_moves_card_idx(self, player_color: PlayerColor, card_idx: int) -> List[Move]:
        return [m for s, m in self.generate_all_legal_moves(player_color) if s == card_idx]  # state.rs:313-320

    def generate_legal_moves(self, player_color: PlayerColor, card: Card) -> List[Move]:  # state.rs:323-378
        slots = [i for i in Deck.get_player_cards_idx(player_color) if self.deck.cards[i] == card]
        return [m for s, m in self.generate_all_legal_moves(player_color) if s in slots]

    def display(self) -> str:  # state.rs:75-108
        border = "---+---+---+---+---+---+\n"
        out = border
        for i in range(25):
            if i % 5 == 0:
                out += f" {5 - i // 5} "
            if get_bit(self.pawns[0], i):
                out += "| r "
            elif get_bit(self.kings[0], i):
                out += "| R "
            elif get_bit(self.pawns[1], i):
                out += "| b "
            elif get_bit(self.kings[1], i):
                out += "| B "
            else:
                out += "| . "
            if (i + 1) % 5 == 0:
                out += "|\n" + border
        return out + "   | a | b | c | d | e |"


def movegen_batch(states: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """oaz_movegen over a STATE_DTYPE array: (moves [n,40] MOVE_DTYPE, counts [n])."""
    states = np.ascontiguousarray(states, dtype=_abi.STATE_DTYPE)
    n = len(states)
    moves = np.zeros((n, _abi.MAX_MOVES), dtype=_abi.MOVE_DTYPE)
    counts = np.zeros(n, dtype=np.uint8)
    _abi.check(_abi.load().oaz_movegen(_abi.ptr(states), n, None, _abi.ptr(moves), _abi.ptr(counts)))
    return moves, counts


def movegen_masks_batch(states: np.ndarray) -> np.ndarray:
    states = np.ascontiguousarray(states, dtype=_abi.STATE_DTYPE)
    masks = np.zeros((len(states), 2, 25), dtype=np.uint32)
    _abi.check(_abi.load().oaz_movegen(_abi.ptr(states), len(states), _abi.ptr(masks), None, None))
    return masks


def step_batch(states: np.ndarray, moves: np.ndarray) -> np.ndarray:
    """oaz_step in place (to_move switches); returns MoveResult codes."""
    assert states.flags["C_CONTIGUOUS"] and states.dtype == _abi.STATE_DTYPE
    moves = np.ascontiguousarray(moves, dtype=_abi.MOVE_DTYPE)
    res = np.zeros(len(states), dtype=np.uint8)
    _abi.check(_abi.load().oaz_step(_abi.ptr(states), _abi.ptr(moves), len(states), _abi.ptr(res)))
    return res


def current_state_batch(states: np.ndarray) -> np.ndarray:
    states = np.ascontiguousarray(states, dtype=_abi.STATE_DTYPE)
    res = np.zeros(len(states), dtype=np.uint8)
    _abi.check(_abi.load().oaz_current_state(_abi.ptr(states), len(states), _abi.ptr(res)))
    return res


def encode_batch(states: np.ndarray) -> np.ndarray:
    """create_tensor_from_state (common.rs:26-80) for each state (colour = to_move): [n,21,5,5]."""
    states = np.ascontiguousarray(states, dtype=_abi.STATE_DTYPE)
    planes = np.zeros((len(states), 21, 5, 5), dtype=np.float32)
    _abi.check(_abi.load().oaz_encode(_abi.ptr(states), len(states), _abi.ptr(planes)))
    return planes


def initial_state_np(deck_idx: Sequence[int]) -> np.ndarray:
    a = np.zeros(1, dtype=_abi.STATE_DTYPE)
    d = (C.c_uint8 * 5)(*deck_idx)
    _abi.load().oaz_initial_state(d, _abi.ptr(a))
    return a


@dataclass
class GameState:  # game_state.rs:6-90
    state: State
    history: List[State] = field(default_factory=list)
    curr_agent_idx: int = 0
    curr_player_color: PlayerColor = PlayerColor.Red

    @staticmethod
    def new(seed: int = 20260101, game_id: int = 0) -> "GameState":
        return GameState.with_deck(Deck.default(seed, game_id))

    @staticmethod
    def with_deck(deck: Deck) -> "GameState":  # game_state.rs:37-51
        st = State.with_deck(deck)
        color = st.deck.neutral_card().player_color
        return GameState(st, [], 0 if color == PlayerColor.Red else 1, color)

    def progress(self, done_move: DoneMove) -> MoveResult:  # game_state.rs:68-83
        self.history.append(self.state.clone())
        if done_move.is_pass():
            res = self.state.pass_turn(done_move.used_card_idx)
        else:
            res = self.state.make_move(done_move.mov, self.curr_player_color, done_move.used_card_idx)
        self.curr_agent_idx = (self.curr_agent_idx + 1) % 2
        self.curr_player_color = self.curr_player_color.enemy()
        return res

    def undo(self) -> None:  # game_state.rs:85-90
        if self.history:
            self.state = self.history.pop()
        self.curr_agent_idx = (self.curr_agent_idx + 1) % 2
        self.curr_player_color = self.curr_player_color.enemy()
