"""Test infrastructure: the reference node's DB layer on real SQLAlchemy (2.0, importable here) over
SQLite, under the bookkeeping of tests/fake_node.py.

* tables with the reference's columns: ``Cycle`` (``cycles/cycle.py:15-25``), ``WorkerCycle``
  (``cycles/worker_cycle.py:20-27``, ``diff = LargeBinary``), ``Model`` / ``ModelCheckPoint``
  (``models/ai_model.py:18-45``), ``Worker`` (``workers/worker.py:17-21``); foreign keys to tables
  the cycle path never reads (fl_process) are left out;
* ``Model.query`` is a thread-scoped session's query property, as Flask-SQLAlchemy 2.4 gives the
  node (one session per thread / greenlet: the executor's close has its own, and reads what the
  handler threads committed);
* ``SqlWarehouse``: ``core/warehouse.py:7-92`` -- ``register`` adds and commits, ``query`` is
  ``filter_by().all()`` (no ORDER BY), ``last`` orders by id desc, ``count`` is
  ``session.query(func.count(id)).filter_by()``, ``modify`` is a bulk ``update`` + commit;
* ``HeapPool``: ``pygrid_amd.report.PinnedPool``'s hand-out / give-back protocol over ordinary
  memory, for CPU runs (page-locked blocks need a GPU); the views it yields are what the installed
  report handler binds into the ``LargeBinary`` column.

Never a product path: only tests import this."""
from __future__ import annotations

import ctypes as C
import threading

from sqlalchemy import Boolean, Column, DateTime, Float, ForeignKey, Integer, LargeBinary, String, create_engine, func
from sqlalchemy.orm import declarative_base, relationship, scoped_session, sessionmaker
from sqlalchemy.pool import StaticPool

from fake_node import make_node
from pygrid_amd.report import PinnedPool, _Return


class SqlStore:
    """One node's database: fresh metadata per store, so tests never share tables."""

    def __init__(self, url: str):
        # "sqlite://" (in memory): one connection shared by every thread, or each would see its own DB
        pool = {"poolclass": StaticPool} if url == "sqlite://" else {}
        self.engine = create_engine(url, connect_args={"check_same_thread": False, "timeout": 30}, **pool)
        self.session = scoped_session(sessionmaker(bind=self.engine), scopefunc=threading.get_ident)
        Base = declarative_base()
        Base.query = self.session.query_property()

        class Worker(Base):
            __tablename__ = "model_centric_worker"
            id = Column(String(255), primary_key=True)
            ping = Column(Float)
            avg_download = Column(Float)
            avg_upload = Column(Float)
            worker_cycle = relationship("WorkerCycle", backref="worker")

        class Cycle(Base):
            __tablename__ = "model_centric_cycle"
            id = Column(Integer, primary_key=True, autoincrement=True)
            start = Column(DateTime())
            end = Column(DateTime())
            sequence = Column(Integer())
            version = Column(String(255))
            worker_cycles = relationship("WorkerCycle", backref="cycle")
            fl_process_id = Column(Integer)
            is_completed = Column(Boolean, default=False)

        class WorkerCycle(Base):
            __tablename__ = "model_centric_worker_cycle"
            id = Column(Integer, primary_key=True, autoincrement=True)
            request_key = Column(String(2048))
            cycle_id = Column(Integer, ForeignKey("model_centric_cycle.id"))
            worker_id = Column(String(255), ForeignKey("model_centric_worker.id"))
            started_at = Column(DateTime())
            is_completed = Column(Boolean(), default=False)
            completed_at = Column(DateTime())
            diff = Column(LargeBinary)

        class Model(Base):
            __tablename__ = "model_centric_model"
            id = Column(Integer, primary_key=True, autoincrement=True)
            version = Column(String(255))
            checkpoints = relationship("ModelCheckPoint", backref="model")
            fl_process_id = Column(Integer, unique=True)

        class ModelCheckPoint(Base):
            __tablename__ = "model_centric_model_checkpoint"
            id = Column(Integer, primary_key=True, autoincrement=True)
            value = Column(LargeBinary)
            number = Column(Integer)
            alias = Column(String(255))
            model_id = Column(Integer, ForeignKey("model_centric_model.id"))

        Base.metadata.create_all(self.engine)
        self.Worker, self.Cycle, self.WorkerCycle = Worker, Cycle, WorkerCycle
        self.Model, self.ModelCheckPoint = Model, ModelCheckPoint
        self.tables = {"model": Model, "checkpoint": ModelCheckPoint, "cycle": Cycle, "worker_cycle": WorkerCycle}

    def warehouse(self, name: str) -> "SqlWarehouse":
        return SqlWarehouse(self, self.tables[name])

    def add_worker(self, worker_id: str):
        self.session.add(self.Worker(id=worker_id))
        self.session.commit()

    def fresh_session(self):
        """A session of its own (nothing cached): what another process would read."""
        return sessionmaker(bind=self.engine)()

    def close(self):
        self.session.remove()
        self.engine.dispose()


class SqlWarehouse:
    def __init__(self, store: SqlStore, schema):
        self._store = store
        self._schema = schema

    @property
    def _session(self):
        return self._store.session

    def register(self, **kwargs):
        obj = self._schema(**kwargs)
        self._session.add(obj)
        self._session.commit()
        return obj

    def query(self, **kwargs):
        return self._schema.query.filter_by(**kwargs).all()

    def count(self, **kwargs):
        return int(self._session.query(func.count(self._schema.id)).filter_by(**kwargs).scalar())

    def first(self, **kwargs):
        return self._schema.query.filter_by(**kwargs).first()

    def last(self, **kwargs):
        return self._schema.query.filter_by(**kwargs).order_by(self._schema.id.desc()).first()

    def modify(self, query, values):
        self._schema.query.filter_by(**query).update(values)
        self._session.commit()

    def update(self):
        self._session.commit()


def make_sql_node(url: str):
    """(node module namespace as tests/fake_node.make_node, its SqlStore)."""
    store = SqlStore(url)
    return make_node(warehouse=store.warehouse), store


class HeapPool(PinnedPool):
    """PinnedPool's protocol over ordinary memory (CPU runs).  ``outstanding`` = blocks handed out
    and not yet given back (a view still referenced somewhere)."""

    def __init__(self, max_blocks: int = 4):
        super().__init__(max_blocks=max_blocks)
        self._mem = {}

    def acquire(self, n: int):
        with self._lock:
            if self._closed or n <= 0 or n > self.max_block_bytes:
                self.misses += 1
                return None
            fits = [b for b in self._free if b[0] >= n]
            if fits:
                cap, addr = min(fits)
                self._free.remove((cap, addr))
            elif self._n < self.max_blocks:
                cap = n
                buf = (C.c_uint8 * cap)()
                addr = C.addressof(buf)
                self._mem[addr] = buf
                self._n += 1
            else:
                self.misses += 1
                return None
            self.hits += 1
        arr = (C.c_uint8 * n).from_address(addr)
        arr._pgh_block = _Return(self, addr, cap)
        return arr, addr

    def _give(self, addr: int, cap: int):
        with self._lock:
            self._free.append((cap, addr))

    @property
    def outstanding(self) -> int:
        return self._n - len(self._free)

    def close(self):
        with self._lock:
            self._closed = True
