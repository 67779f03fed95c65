"""Write tests/golden/reference_kats.json: the reference's own known-answer tests for the hot
path, transcribed as data (inputs + expected outputs) from the Rust unit tests.

Sources (paths relative to the reference root):
  onitama-game/src/game/state.rs:381-890     rules tests
  onitama-game/src/common/mod.rs:77-135      bit-order tests
  onitama-game/src/ai/mcts/mcts_arena.rs:403-457  exact child (expansion) order fixtures
  onitama-game/src/ai/mcts/mcts_arena.rs:459-554  tactical positions (pure-MCTS sanity tests)
Run: python tools/make_reference_kats.py
"""
import json
from pathlib import Path

# card indices (card.rs:465-468)
TIGER, DRAGON, FROG, RABBIT, CRAB, ELEPHANT, GOOSE, ROOSTER, MONKEY, MANTIS, CRANE, HORSE, OX, BOAR, EEL, COBRA = range(16)
P, K = 0, 1
RED, BLUE = 0, 1
CAPTURE, RED_WIN, BLUE_WIN, IN_PROGRESS = 0, 1, 2, 3
RK, BK, RP, BP = 0x0000_0200, 0x2000_0000, 0x0000_0D80, 0xD800_0000


def sq(r, c):
    return r * 5 + c


def bb(r, c):  # from_2d_to_bitboard
    return 0x8000_0000 >> sq(r, c)


def start(deck, kings=(RK, BK), pawns=(RP, BP)):
    return {"deck": deck, "kings": list(kings), "pawns": list(pawns)}


movegen = [
    {"src": "state.rs:419-454 create_all_legal_moves_for_red_in_starting_position",
     "state": start([CRAB, RABBIT, DRAGON, TIGER, FROG]), "color": RED, "slot": 0,
     "moves": [[sq(4, 0), sq(3, 0), P], [sq(4, 1), sq(3, 1), P], [sq(4, 2), sq(3, 2), K],
               [sq(4, 3), sq(3, 3), P], [sq(4, 4), sq(3, 4), P]]},
    {"src": "state.rs:419-454 (rabbit)", "state": start([CRAB, RABBIT, DRAGON, TIGER, FROG]), "color": RED,
     "slot": 1, "moves": [[sq(4, 0), sq(3, 1), P], [sq(4, 1), sq(3, 2), P], [sq(4, 2), sq(3, 3), K],
                          [sq(4, 3), sq(3, 4), P]]},
    {"src": "state.rs:456-492 create_all_legal_moves_for_blue_in_starting_position",
     "state": start([DRAGON, TIGER, CRAB, RABBIT, FROG]), "color": BLUE, "slot": 2,
     "moves": [[sq(0, 0), sq(1, 0), P], [sq(0, 1), sq(1, 1), P], [sq(0, 2), sq(1, 2), K],
               [sq(0, 3), sq(1, 3), P], [sq(0, 4), sq(1, 4), P]]},
    {"src": "state.rs:456-492 (rabbit)", "state": start([DRAGON, TIGER, CRAB, RABBIT, FROG]), "color": BLUE,
     "slot": 3, "moves": [[sq(0, 1), sq(1, 0), P], [sq(0, 2), sq(1, 1), K], [sq(0, 3), sq(1, 2), P],
                          [sq(0, 4), sq(1, 3), P]]},
    {"src": "state.rs:818-850 blue_to_move_no_legal_moves",
     "state": start([DRAGON, TIGER, RABBIT, HORSE, FROG], kings=(512, 67108864), pawns=(61568, 3221225472)),
     "color": BLUE, "slot": 2, "moves": []},
    {"src": "state.rs:852-889 no_legal_moves_at_all_pass_is_required (tiger)",
     "state": start([DRAGON, RABBIT, TIGER, HORSE, FROG], kings=(16384, 131072), pawns=(2148009984, 138416256)),
     "color": BLUE, "slot": 2, "moves": []},
    {"src": "state.rs:852-889 (horse)",
     "state": start([DRAGON, RABBIT, TIGER, HORSE, FROG], kings=(16384, 131072), pawns=(2148009984, 138416256)),
     "color": BLUE, "slot": 3, "moves": []},
]

make_move = [
    {"src": "state.rs:494-518 make_move_as_red", "state": start([CRAB, RABBIT, DRAGON, TIGER, FROG]),
     "move": [20, 15, P, 0], "color": RED, "result": IN_PROGRESS,
     "bits": [["pawns", RED, 15, 1], ["pawns", RED, 20, 0]], "neutral": CRAB},
    {"src": "state.rs:520-544 make_move_as_blue", "state": start([CRAB, RABBIT, DRAGON, TIGER, FROG]),
     "move": [1, 11, P, 3], "color": BLUE, "result": IN_PROGRESS,
     "bits": [["pawns", BLUE, 11, 1], ["pawns", BLUE, 1, 0]], "neutral": TIGER},
    {"src": "state.rs:546-589 capture_as_red",
     "state": start([CRAB, RABBIT, DRAGON, TIGER, FROG], pawns=(RP, 0x5801_0000)),
     "move": [20, 15, P, 0], "color": RED, "result": CAPTURE,
     "bits": [["pawns", RED, 15, 1], ["pawns", RED, 20, 0]], "neutral": CRAB, "equals": [["pawns", BLUE, 0x5800_0000]]},
    {"src": "state.rs:591-634 capture_as_blue",
     "state": start([CRAB, RABBIT, DRAGON, TIGER, FROG], pawns=(RP, 0x5820_0000)),
     "move": [10, 20, P, 3], "color": BLUE, "result": CAPTURE,
     "bits": [["pawns", BLUE, 20, 1], ["pawns", BLUE, 10, 0]], "neutral": TIGER, "equals": [["pawns", RED, 0x0000_0580]]},
    {"src": "state.rs:636-679 capture_win_as_red",
     "state": start([CRAB, RABBIT, DRAGON, TIGER, FROG], pawns=(0x0100_0680, BP)),
     "move": [7, 2, P, 0], "color": RED, "result": RED_WIN,
     "bits": [["pawns", RED, 2, 1], ["pawns", RED, 7, 0]], "neutral": CRAB, "equals": [["kings", BLUE, 0]]},
    {"src": "state.rs:681-724 capture_win_as_blue",
     "state": start([CRAB, RABBIT, DRAGON, TIGER, FROG], pawns=(RP, 0x5808_0000)),
     "move": [12, 22, P, 3], "color": BLUE, "result": BLUE_WIN,
     "bits": [["pawns", BLUE, 22, 1], ["pawns", BLUE, 12, 0]], "neutral": TIGER, "equals": [["kings", RED, 0]]},
    {"src": "state.rs:726-770 king_in_temple_as_blue",
     "state": start([CRAB, RABBIT, DRAGON, TIGER, FROG], kings=(0x0000_2000, 0x0008_0000)),
     "move": [12, 22, K, 3], "color": BLUE, "result": BLUE_WIN,
     "bits": [["kings", BLUE, 22, 1], ["kings", BLUE, 12, 0]], "neutral": TIGER, "nonzero": [["kings", RED]]},
    {"src": "state.rs:772-816 king_in_temple_as_red",
     "state": start([CRAB, RABBIT, DRAGON, TIGER, FROG], kings=(0x0100_0000, 0x0008_0000)),
     "move": [7, 2, K, 0], "color": RED, "result": RED_WIN,
     "bits": [["kings", RED, 2, 1], ["kings", RED, 7, 0]], "neutral": CRAB, "nonzero": [["kings", BLUE]]},
]

bits = {
    "src": "common/mod.rs:77-135",
    "get_bit": {"value": 0b0000_1111_0000_1111_0000_1111_0000_1111,
                "expected": [0, 0, 0, 0, 1, 1, 1, 1] * 4},
    "from_2d_to_bitboard": [[[0, 0], 0x8000_0000], [[2, 1], 0x0010_0000], [[4, 4], 0x0000_0080]],
}

display = {
    "src": "state.rs:397-417 correct_display",
    "expected": ("---+---+---+---+---+---+\n 5 | b | b | B | b | b |\n---+---+---+---+---+---+\n"
                 " 4 | . | . | . | . | . |\n---+---+---+---+---+---+\n 3 | . | . | . | . | . |\n"
                 "---+---+---+---+---+---+\n 2 | . | . | . | . | . |\n---+---+---+---+---+---+\n"
                 " 1 | r | r | R | r | r |\n---+---+---+---+---+---+\n   | a | b | c | d | e |"),
}

expansion = [
    {"src": "onitama-game/src/ai/mcts/mcts_arena.rs:403-423 test_first_expand_debug_print",
     "state": start([DRAGON, FROG, TIGER, RABBIT, HORSE]), "color": RED,
     "children": ["Dragon a1-c2", "Dragon b1-d2", "Dragon c1-a2", "Dragon c1-e2", "Dragon d1-b2",
                  "Dragon e1-c2", "Frog b1-a2", "Frog c1-b2", "Frog d1-c2", "Frog e1-d2"]},
    {"src": "onitama-game/src/ai/mcts/mcts_arena.rs:425-457 test_root_child_expand_debug_print",
     "state": start([DRAGON, FROG, TIGER, RABBIT, HORSE]), "color": BLUE,
     "children": ["Tiger a5-a3", "Tiger b5-b3", "Tiger c5-c3", "Tiger d5-d3", "Tiger e5-e3",
                  "Rabbit b5-a4", "Rabbit c5-b4", "Rabbit d5-c4", "Rabbit e5-d4"]},
]

# Pure-MCTS tactical sanity tests (stochastic in the reference, 1 s wall-clock rollouts); the
# expected move is a forced tactical answer, used here as an AZ-search sanity check.
tactics = [
    {"src": "onitama-game/src/ai/mcts/mcts_arena.rs:459-483 test_best_move_win",
     "state": start([RABBIT, FROG, TIGER, DRAGON, HORSE], kings=(bb(1, 3), BK)), "color": BLUE,
     "expected": [1, 8, P, 3]},
    {"src": "onitama-game/src/ai/mcts/mcts_arena.rs:485-517 test_no_way_to_hide_for_blue",
     "state": start([OX, MONKEY, RABBIT, HORSE, DRAGON], kings=(RK, bb(0, 4)),
                    pawns=(bb(0, 3) | bb(1, 4), 0)), "color": BLUE, "expected": [4, 2, K, 2]},
    {"src": "onitama-game/src/ai/mcts/mcts_arena.rs:519-553 test_worst_case_capture_blue",
     "state": start([MONKEY, ROOSTER, GOOSE, MANTIS, HORSE], kings=(RK, bb(1, 2)),
                    pawns=(bb(2, 3) | bb(3, 2), BP)), "color": BLUE, "expected": [7, 2, K, 3]},
]

out = {"movegen": movegen, "make_move": make_move, "bits": bits, "display": display,
       "expansion": expansion, "tactics": tactics}
path = Path(__file__).resolve().parents[1] / "tests" / "golden" / "reference_kats.json"
path.write_text(json.dumps(out, indent=1))
print("wrote", path)
