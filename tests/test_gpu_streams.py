"""GPU: engine and trainer creation are ordered on their own streams.

Round 5 saw a concurrent-creation flake: creation zeroed the counters with null-stream hipMemsets, which
the engine's non-blocking streams do not wait for, so a late memset could land after the first move's
sample count (fixed in 08b85c8: creation zeroes and uploads on the engine's own stream and waits). This is
the deterministic regression test of that cause: the legacy null stream is kept busy by a spin kernel
while an engine (then a trainer) is created and used, and every result must equal a quiet run's, byte
for byte. The test also checks that the window was open: the engine's whole run finished while the null
stream was still spinning."""
import numpy as np
import pytest
import torch

from onitama_az import _abi
from onitama_az.engine import Engine
from onitama_az.weights import random_weights

pytestmark = pytest.mark.gpu

KW = dict(games=64, sims=16, c_puct=5.0, train_noise=1, evaluator=_abi.EVAL_HASH, blocks=0, max_plies=150, seed=77,
          fixed_deck=0)


def _spin_null_stream(seconds):
    """A spin kernel of about `seconds` on torch's current stream, which in this process is the legacy
    null stream; returns an event recorded behind it."""
    assert torch.cuda.current_stream().cuda_stream == 0, "torch's current stream is not the null stream"
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    cycles = 1 << 22
    a.record()
    torch.cuda._sleep(cycles)
    b.record()
    b.synchronize()
    per_cycle_ms = a.elapsed_time(b) / cycles
    torch.cuda._sleep(int(seconds * 1e3 / max(per_cycle_ms, 1e-9)))
    done = torch.cuda.Event()
    done.record()
    return done


def _selfplay(done=None):
    """Create an engine, play 40 plies, read the statistics and the records back; `open` = the null stream
    was still spinning when all that had finished (before the engine's hipFree, which waits for the device)."""
    with Engine(**KW) as e:
        e.selfplay_reset()
        e.selfplay_step(40)
        st = e.selfplay_stats()
        smp = e.samples_fetch(1 << 16)
        still_busy = done is not None and not done.query()
    key = (st.moves, st.games_finished, st.games_cut, st.red_wins, st.blue_wins, st.samples_ready, st.samples_dropped,
           st.passes, st.search.sims, st.search.expansions, st.search.children, st.search.depth_sum, st.search.nn_evals)
    return key, smp, still_busy


def _train(samples, w, done=None):
    from onitama_az.trainer import Trainer
    with Trainer(blocks=1, max_batch=64) as tr:
        tr.set_weights(w)
        tr.load_samples(samples)
        tr.set_batches(np.arange(128, dtype=np.int32).reshape(2, 64))
        tr.train(0, 2)
        out = tr.get_weights(), tr.losses()
        still_busy = done is not None and not done.query()
    return out + (still_busy,)


@pytest.mark.timeout(180)
def test_creation_behind_busy_null_stream_equals_quiet_run():
    torch.cuda.init()
    ref_key, ref, _ = _selfplay()
    assert ref_key[5] > 128 and len(ref) == ref_key[5]
    w = random_weights(3, 1)
    ref_w, ref_loss, _ = _train(ref[:128], w)

    done = _spin_null_stream(3.0)
    key, smp, open_e = _selfplay(done)
    torch.cuda.synchronize()
    done = _spin_null_stream(3.0)
    got_w, got_loss, open_t = _train(ref[:128], w, done)
    torch.cuda.synchronize()
    assert open_e and open_t, ("the run waited for the null stream: the race window was closed", open_e, open_t)
    assert key == ref_key
    assert smp.tobytes() == ref.tobytes()  # the records too, in the same (slot) order
    assert got_w.tobytes() == ref_w.tobytes() and got_loss == ref_loss
