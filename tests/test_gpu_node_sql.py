"""GPU: the installed node on the real engine against the reference's storage types and report
handler -- tests/test_node_sql.py's scenario with MNIST-sized diffs (784-392-10,
1.2 MB State messages: the handler's clean base64 route) decoded into the library's page-locked
blocks (``PinnedPool``), bound into SQLAlchemy's ``LargeBinary`` column, DMA'd to HBM as they lie
(``pgh_ingest_state``) and folded at report time.  The saved checkpoints must be byte-identical to
the reference node's torch close over the same DB rows; every block must come back to its pool."""
import gc

import numpy as np
import pytest

from test_node_sql import CFG, SqlScenario, random_script, run_both, script_three_cycles

pytestmark = pytest.mark.gpu
F = np.float32
MNIST = [(392, 784), (392,), (10, 392), (10,)]


def mnist_ckpt():
    from pygrid_amd.state_schema import build_state_fast

    rng = np.random.default_rng(71)
    return build_state_fast([(rng.standard_normal(s) * 0.05).astype(F) for s in MNIST])


def mnist_diff(worker, version=0):
    import zlib

    from pygrid_amd.state_schema import build_state_fast

    rng = np.random.default_rng([version, zlib.crc32(str(worker).encode()), 72])
    return build_state_fast([(rng.standard_normal(s) * 10.0 ** rng.integers(-4, 0)).astype(F) for s in MNIST])


@pytest.mark.parametrize("slots", [None, 2], ids=["slots-default", "slots-2"])
@pytest.mark.parametrize("threaded", [False, True], ids=["sync", "executor"])
def test_installed_sql_node_with_pinned_reports_on_the_gpu(tmp_path, engine, slots, threaded):
    def fresh_engine():  # a (re)started node process has nothing resident in HBM
        engine.reset()
        engine.ckpt_owner = None
        return engine

    eng = run_both(tmp_path, script_three_cycles, engine=fresh_engine, ckpt=mnist_ckpt(), diff_fn=mnist_diff,
                   threaded=threaded, pinned_reports=4, slots=slots)
    st = eng.stats
    assert st["closes_report_time"] == 3 and st["closes_close_time"] == 0 and st["report_errors"] == 0, st
    gc.collect()
    pools = [(p.hits, p.misses, p.blocks) for p in eng.pools]
    # every report decoded into a page-locked block; every block freed once its views were gone
    assert pools == [(12, 0, 0), (2, 0, 0)], pools
    assert CFG["num_cycles"] == 3


def test_installed_sql_node_on_a_group(tmp_path):
    """The same node on a one-process group of two children sharing GPU 0 (what a node with
    several GPUs installs: ``install(devices=[...])``): each report's payload slices go to their
    child, every child folds its shard, the close frames one checkpoint -- byte-identical to the
    reference node; the page-locked blocks all come back."""
    from pygrid_amd import Engine

    with Engine(devices=[0, 0]) as grp:
        def fresh_group():
            grp.reset()
            grp.ckpt_owner = None
            return grp

        eng = run_both(tmp_path, script_three_cycles, engine=fresh_group, ckpt=mnist_ckpt(), diff_fn=mnist_diff,
                       pinned_reports=4)
        st = eng.stats
        assert st["closes_report_time"] == 3 and st["report_errors"] == 0, st
    gc.collect()
    assert [(p.hits, p.misses, p.blocks) for p in eng.pools] == [(12, 0, 0), (2, 0, 0)]


def test_randomised_scripts_on_the_gpu_sql_node(tmp_path, engine):
    """tests/test_node_sql.py's random scripts on the GPU engine with page-locked report blocks and
    the close on an executor thread: byte-identical checkpoints and DB diffs."""
    def fresh_engine():
        engine.reset()
        engine.ckpt_owner = None
        return engine

    for trial in range(4):
        script, slots = random_script(600 + trial, f"g{trial}")
        eng = run_both(tmp_path / f"t{trial}", script, engine=fresh_engine, ckpt=mnist_ckpt(), diff_fn=mnist_diff,
                       threaded=True, pinned_reports=4, slots=slots)
        st = eng.stats
        assert st["closes_report_time"] == 3 and st["report_errors"] == 0, (trial, st)
