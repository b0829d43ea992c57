"""Checkpoint / resume and fault injection for the elimination loop
(SURVEY.md §5.3-5.4).

The reference keeps its state in process memory only and restarts from
scratch; its pivot loop index is the natural checkpoint boundary.  Here the
boundary is a panel (column block) of the distributed solver: after block g
every rank's state is its local column slab with the replicated b (n x ld
doubles), the zero-pivot flag and g itself.

Protocol (consistent under a crash at any point):
  1. every rank writes `rank{r}_b{g}.safetensors` (tmp file + os.replace);
  2. barrier;
  3. rank 0 atomically replaces `manifest.json` with {"block": g, ...};
  4. barrier; every rank deletes its files of older blocks.
A resume reads the manifest, so a crash between 1 and 3 falls back to the
previous complete generation.  Files are safetensors + JSON: nothing in them
is executed on load.

Fault injection: `GELIM_FAULT_AT_BLOCK=g` (optionally `GELIM_FAULT_RANK=r`)
makes the solver raise `InjectedFault` on entering block g, which is how the
tests kill a run mid-elimination and resume it.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass
from pathlib import Path

import torch


class InjectedFault(RuntimeError):
    """Raised by the fault-injection hook (GELIM_FAULT_AT_BLOCK)."""


def maybe_inject_fault(block: int, rank: int, at: int | None = None) -> None:
    if at is None:
        env = os.environ.get("GELIM_FAULT_AT_BLOCK")
        at = int(env) if env not in (None, "") else None
    if at is None or block != at:
        return
    fr = os.environ.get("GELIM_FAULT_RANK")
    if fr not in (None, "") and int(fr) != rank:
        return
    raise InjectedFault(f"injected fault at block {block} on rank {rank}")


@dataclass
class CheckpointState:
    block: int            # first block NOT yet processed
    loc: torch.Tensor     # local slab (CPU)
    info: torch.Tensor    # zero-pivot flags (CPU)


class Checkpointer:
    """Panel-boundary checkpoints of one distributed solve (see module doc)."""

    def __init__(self, directory: str | os.PathLike, comm, meta: dict, every: int = 1):
        if every < 1:
            raise ValueError("checkpoint interval must be >= 1 block")
        self.dir = Path(directory)
        self.comm = comm
        self.meta = {k: str(v) for k, v in meta.items()}
        self.every = every
        self.dir.mkdir(parents=True, exist_ok=True)

    def _file(self, block: int) -> Path:
        return self.dir / f"rank{self.comm.rank}_b{block}.safetensors"

    def due(self, next_block: int) -> bool:
        return next_block % self.every == 0

    def save(self, next_block: int, loc: torch.Tensor, info: torch.Tensor) -> None:
        from safetensors.torch import save_file

        f = self._file(next_block)
        tmp = f.with_suffix(".tmp")
        meta = dict(self.meta, block=str(next_block), rank=str(self.comm.rank))
        save_file({"loc": loc.detach().cpu().contiguous(), "info": info.detach().cpu().contiguous()},
                  str(tmp), metadata=meta)
        os.replace(tmp, f)
        self.comm.barrier()
        if self.comm.rank == 0:
            man = self.dir / "manifest.json"
            tmpm = man.with_suffix(".tmp")
            tmpm.write_text(json.dumps(dict(self.meta, block=next_block, world_size=self.comm.world_size)))
            os.replace(tmpm, man)
        self.comm.barrier()
        for old in self.dir.glob(f"rank{self.comm.rank}_b*.safetensors"):
            if old != f:
                old.unlink(missing_ok=True)

    def load(self) -> CheckpointState | None:
        """The last complete generation for this rank, or None."""
        from safetensors import safe_open

        man = self.dir / "manifest.json"
        if not man.exists():
            return None
        m = json.loads(man.read_text())
        if int(m["world_size"]) != self.comm.world_size:
            raise ValueError(f"checkpoint written by {m['world_size']} ranks, resuming with {self.comm.world_size}")
        f = self._file(int(m["block"]))
        with safe_open(str(f), framework="pt") as fh:
            fm = fh.metadata()
            for k, v in self.meta.items():  # per-rank metadata (ld differs by rank)
                if fm.get(k) != v:
                    raise ValueError(f"checkpoint {k}={fm.get(k)} does not match this solve ({v})")
            if int(fm["block"]) != int(m["block"]) or int(fm["rank"]) != self.comm.rank:
                raise ValueError(f"{f} does not belong to manifest block {m['block']}")
            return CheckpointState(int(m["block"]), fh.get_tensor("loc"), fh.get_tensor("info"))

    def clear(self) -> None:
        self.comm.barrier()
        for f in self.dir.glob(f"rank{self.comm.rank}_b*.safetensors"):
            f.unlink(missing_ok=True)
        self.comm.barrier()
        if self.comm.rank == 0:
            (self.dir / "manifest.json").unlink(missing_ok=True)
