"""CPU: checkpoint store mirrors ModelManager.save/load numbering and the latest alias
(model_manager.py:30-60) and /retrieve-model's selection (routes.py:488-498)."""
import pytest

from pygrid_amd.checkpoints import CheckpointStore, ModelNotFoundError


def test_numbering_and_latest_alias():
    st = CheckpointStore()
    st.create(1, b"c1")
    st.save(1, b"c2")
    st.save(2, b"other")
    cp = st.save(1, b"c3")
    assert cp.number == 3 and cp.alias == "latest"
    assert st.latest(1) == b"c3"
    assert st.retrieve(1) == b"c3"
    assert st.retrieve(1, "1") == b"c1"
    assert st.retrieve(1, "2") == b"c2"
    assert st.retrieve(1, "latest") == b"c3"
    assert [c.alias for c in st._by_model[1]] == ["", "", "latest"]
    assert st.latest(2) == b"other"


def test_missing_raises_model_not_found():
    st = CheckpointStore()
    with pytest.raises(ModelNotFoundError):
        st.latest(7)
    st.create(7, b"x")
    with pytest.raises(ModelNotFoundError):
        st.retrieve(7, "9")
    with pytest.raises(ModelNotFoundError):
        st.retrieve(7, "best")


def test_store_returns_the_same_object_for_resident_reuse():
    st = CheckpointStore()
    blob = bytes(1000)
    st.save(3, blob)
    assert st.latest(3) is blob  # CycleAggregator reuses the HBM copy on identity


def test_invalidate_and_cached_bytes():
    """``invalidate`` (one model or all) makes the next lookup fall through to the DB; ``keep``
    bounds what ``cached_bytes`` counts."""
    st = CheckpointStore(keep=2)
    for k in range(4):
        st.save(1, bytes(100 + k))
    st.save(2, bytes(50))
    assert st.cached_bytes == 102 + 103 + 50  # model 1 keeps its newest two
    assert st.lookup(model_id=1, alias="latest").value == bytes(103)
    st.invalidate(1)
    assert st.lookup(model_id=1) is None and st.lookup(model_id=2).value == bytes(50)
    assert st.cached_bytes == 50
    st.invalidate()
    assert st.cached_bytes == 0 and st.lookup(model_id=2) is None
