"""Tile-state checkpoints: Spark's state store behind checkpointLocation (reference heatmap_stream.py:37,244).

Spark keeps the aggregation state under the query's checkpointLocation and, after a restart, re-runs the first
uncommitted epoch on the state of the epoch before it.  Here every rank (one GPU, one engine) keeps a chain of files
under ``<CHECKPOINT>/mobheat-state``, like Spark's HDFS state store: a full snapshot (``state-<E>``), then one delta per
committed epoch (``delta-<E>``: the keys that epoch touched, hm_state_export_touched), a new snapshot every
``full_every`` deltas.  File names carry the rank and the world size: ``state-<E>.r<rank>of<world>.mhs`` (a JSON
header and the raw records, engine.save_state_file; ``.npz`` files of earlier versions are read too).

Every file records, besides the engine's state (hm_state_info + 64-B records), its chain: the lineage id (one per
uninterrupted stream of epochs: a fresh stream starts a new one), the epoch of the chain's snapshot and of the file
before it.  A restore follows those links back from the newest epoch before the replayed one and uses a chain only if
it is unbroken and every rank of its world has one ending at that same epoch; files that belong to no such chain (an
abandoned lineage, an older query's leftovers) are never merged into the state.  Saving epoch E first
deletes the rank's files of epochs >= E: Spark re-running E abandons whatever was written after it.

A restore into another world size (N GPUs -> M) loads every old rank's chain and keeps the keys the new rank owns
(``distributed.tile_owner``): ownership is a pure function of the key, so the union of the new ranks' states is the old
state exactly.
"""
import json
import os
import re
import uuid
import warnings
from collections import namedtuple

import numpy as np

Entry = namedtuple("Entry", "epoch kind rank world path")
_NAME = re.compile(r"^(state|delta)-(-?\d+)(?:\.r(\d+)of(\d+))?\.(?:mhs|npz)$")
RestorePoint = namedtuple("RestorePoint", "epoch world lineage")
LEGACY = "legacy"   # the lineage of files written before chains were recorded (no meta)


def new_lineage():
    return uuid.uuid4().hex


class StateCheckpoints:
    """The checkpoint files of one rank of a `world`-rank stream under `root` (the state directory)."""

    def __init__(self, root, rank=0, world=1):
        self.root = root
        self.rank = int(rank)
        self.world = int(world)
        self._meta_cache = {}

    # ---- files ----
    def scan(self):
        """Every checkpoint file under root: [Entry], sorted by (epoch, rank)."""
        if not os.path.isdir(self.root):
            return []
        out = []
        for name in os.listdir(self.root):
            m = _NAME.match(name)
            if not m:
                continue
            kind = "full" if m.group(1) == "state" else "delta"
            rank = int(m.group(3)) if m.group(3) is not None else 0
            world = int(m.group(4)) if m.group(4) is not None else 1
            out.append(Entry(int(m.group(2)), kind, rank, world, os.path.join(self.root, name)))
        return sorted(out, key=lambda e: (e.epoch, e.rank, e.world))

    def path(self, kind, epoch, rank=None, world=None):
        rank = self.rank if rank is None else rank
        world = self.world if world is None else world
        return os.path.join(self.root, f"{'state' if kind == 'full' else 'delta'}-{int(epoch)}.r{rank}of{world}.mhs")

    def _raw_meta(self, e):
        key = (e.path, os.path.getmtime(e.path) if os.path.exists(e.path) else 0)
        if key not in self._meta_cache:
            from .engine import read_state_meta
            try:
                raw = read_state_meta(e.path)
                m = json.loads(raw) if raw is not None else None
            except (OSError, ValueError, KeyError, RuntimeError):
                m = None
            self._meta_cache[key] = m
        return self._meta_cache[key]

    def meta(self, e):
        """The chain record of a file: lineage, base (its snapshot's epoch), prev (the file before it, -1 for a
        snapshot).  Files without one -- the ``state-<E>.npz`` / ``delta-<E>.npz`` files of the version before chains
        were recorded -- follow that version's rule: a legacy delta continues the legacy file of its rank just
        before it, on the newest legacy snapshot before it, all in one lineage "legacy"; a stream restored from them
        continues that lineage."""
        m = self._raw_meta(e)
        if m is not None:
            return m
        if e.kind == "full":
            return {"lineage": LEGACY, "base": e.epoch, "prev": -1}
        older = [x for x in self.scan() if x.rank == e.rank and x.world == e.world and x.epoch < e.epoch
                 and self._raw_meta(x) is None]
        if not older:
            return {"lineage": LEGACY, "base": None, "prev": None}
        prev = older[-1].epoch
        fulls = [x.epoch for x in older if x.kind == "full"]
        return {"lineage": LEGACY, "base": fulls[-1] if fulls else None, "prev": prev}

    # ---- chains ----
    def chain_to(self, rank, world, epoch, entries=None):
        """The chain of (rank, world) ending at its file of `epoch`: [Entry] from the snapshot to that file, or None
        when there is no such file or its chain is broken (a missing link, or a link of another lineage)."""
        entries = self.scan() if entries is None else entries
        mine = {e.epoch: e for e in entries if e.rank == rank and e.world == world and e.epoch <= epoch}
        if epoch not in mine:
            return None
        last = mine[epoch]
        lineage = self.meta(last)["lineage"]
        out = [last]
        while out[-1].kind != "full":
            prev = self.meta(out[-1])["prev"]
            e = mine.get(prev) if prev is not None and prev < out[-1].epoch else None
            if e is None or self.meta(e)["lineage"] != lineage:
                return None
            out.append(e)
        return out[::-1]

    def restore_point(self, before):
        """The newest epoch C < `before` at which some world W has an unbroken chain for every one of its ranks, all
        ending at C in one lineage: RestorePoint(C, W, lineage), or None.  Warns when files exist but none qualifies
        (the stream then starts from an empty state, as a new query would)."""
        entries = self.scan()
        if not entries:
            return None
        best = None
        for world in sorted({e.world for e in entries}):
            for C in sorted({e.epoch for e in entries if e.world == world and e.epoch < before}, reverse=True):
                if best is not None and C < best.epoch:
                    break
                chains = [self.chain_to(r, world, C, entries) for r in range(world)]
                if any(c is None for c in chains):
                    continue
                lineages = {self.meta(c[-1])["lineage"] for c in chains}
                if len(lineages) != 1:
                    continue
                cand = RestorePoint(C, world, lineages.pop())
                if best is None or C > best.epoch or world == self.world:
                    best = cand
                break
        if best is None and any(e.epoch < before for e in entries):
            warnings.warn(f"mobheat: state checkpoints exist under {self.root} but no complete chain ends before epoch "
                          f"{before}; starting from an empty state", RuntimeWarning, stacklevel=2)
        return best

    def load(self, point, owner=None):
        """The state at a restore point: (info, records) merged from the snapshot + deltas of every rank of its world;
        with `owner` (a function of (cell, window_start_us) -> bool) only the keys it selects."""
        from .engine import load_state_file, merge_state
        entries = self.scan()
        same = point.world == self.world   # (the same world: the same owners, this rank's own chain holds its keys)
        ranks = [self.rank] if same else range(point.world)
        infos, parts = [], []
        for r in ranks:
            ch = self.chain_to(r, point.world, point.epoch, entries)
            if ch is None:
                raise RuntimeError(f"mobheat: the checkpoint chain of rank {r} of {point.world} changed under the restore")
            info, recs = merge_state(load_state_file(ch[0].path), [load_state_file(e.path) for e in ch[1:]])
            infos.append(info)
            if not same and owner is not None and recs.size:
                recs = recs[owner(recs["cell"], recs["window_start_us"])]
            parts.append(recs)
        recs = np.concatenate(parts) if len(parts) > 1 else parts[0]
        info = dict(infos[0], n_keys=int(recs.size))
        return info, np.ascontiguousarray(recs)

    # ---- save ----
    def save(self, epoch, engine, lineage, full_every):
        """Checkpoint the engine's state after epoch `epoch` into this rank's chain of `lineage` (prepare + write)."""
        return self.write(self.prepare(epoch, engine, lineage, full_every))

    def prepare(self, epoch, engine, lineage, full_every):
        """The engine's part of a checkpoint of epoch `epoch` (call it from the engine's thread, before the next batch
        changes the state): a snapshot when this rank's chain of `lineage` has none or `full_every` deltas followed
        the newest one, else the epoch's delta (hm_state_export_touched), copied to host memory.  Returns the job
        write() finishes -- the file I/O, which may run on another thread (foreach_batch_func overlaps it with the
        sink's writes)."""
        epoch = int(epoch)
        entries = [e for e in self.scan() if not (e.rank == self.rank and e.world == self.world and e.epoch >= epoch)]
        ch = None   # this rank's chain of `lineage` ending at its newest epoch before `epoch`
        for C in sorted({e.epoch for e in entries if e.rank == self.rank and e.world == self.world}, reverse=True):
            c = self.chain_to(self.rank, self.world, C, entries)
            if c is not None and self.meta(c[-1])["lineage"] == lineage:
                ch = c
            break
        # (the records: a view of the engine's page-locked export buffer, valid until its next export -- the caller
        # writes the file before the next batch: foreach_batch_func and the sharded writer wait for it)
        full = ch is None or len(ch) - 1 >= int(full_every)
        if full:
            meta = {"lineage": lineage, "base": epoch, "prev": -1, "rank": self.rank, "world": self.world}
        else:
            meta = {"lineage": lineage, "base": ch[0].epoch, "prev": ch[-1].epoch, "rank": self.rank,
                    "world": self.world}
        job = {"epoch": epoch, "kind": "full" if full else "delta", "meta": meta, "fill": None, "raw": None}
        if hasattr(engine, "export_begin"):
            # only the dump here (~1 ms per 1e7 keys); the device-to-host copy runs in write(), slice by slice beside
            # the file's writes -- and beside the statements' encode, which the caller starts meanwhile
            job["info"], _, job["recs"], job["raw"], job["fill"] = engine.export_begin(touched_only=not full)
        else:
            job["info"], job["recs"] = engine.export_state(reuse=True) if full else engine.export_state_delta(reuse=True)
        return job

    def write(self, job):
        """The file side of a prepared checkpoint: this rank's files of epochs >= its epoch deleted (an abandoned
        lineage), the file written atomically (fsync + rename), then every file of this rank that the newest two
        snapshots of the chain no longer need (other lineages included).  Returns the kind written."""
        import time
        from .engine import save_state_file
        t0 = time.perf_counter()
        epoch = job["epoch"]
        os.makedirs(self.root, exist_ok=True)
        for e in self.scan():
            if e.rank == self.rank and e.world == self.world and e.epoch >= epoch:
                _remove(e.path)
        t1 = time.perf_counter()
        stats = save_state_file(self.path(job["kind"], epoch), job["info"], job["recs"], meta=json.dumps(job["meta"]),
                                fill=job.get("fill"), raw=job.get("raw"))
        t2 = time.perf_counter()
        self._prune(job["meta"]["lineage"], epoch)
        # (the file side's phases, ms: foreach_batch_func reports them beside its own)
        job["timings"] = {"ckpt_clear": 1e3 * (t1 - t0), "ckpt_file": 1e3 * (t2 - t1),
                          "ckpt_prune": 1e3 * (time.perf_counter() - t2), **stats}
        return job["kind"]

    def _prune(self, lineage, epoch):
        mine = [e for e in self.scan() if e.rank == self.rank and e.world == self.world]
        fulls = [e for e in mine if e.kind == "full" and self.meta(e)["lineage"] == lineage]
        keep_from = fulls[-2].epoch if len(fulls) >= 2 else (fulls[0].epoch if fulls else epoch)
        for e in mine:
            if e.epoch < keep_from or self.meta(e)["lineage"] != lineage:
                _remove(e.path)


    def prune_other_worlds(self, lineage):
        """Delete the files of other world sizes once every rank of this world has a snapshot of `lineage` (called by
        the coordinator after a commit: a restore can then always use this world's chains)."""
        entries = self.scan()
        for r in range(self.world):
            if not any(e.rank == r and e.world == self.world and e.kind == "full" and self.meta(e)["lineage"] == lineage
                       for e in entries):
                return
        for e in entries:
            if e.world != self.world:
                _remove(e.path)


def _remove(path):
    try:
        os.remove(path)
    except FileNotFoundError:
        pass
