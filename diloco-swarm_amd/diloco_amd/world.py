"""Process topology for the outer step (src/world.py:10-119): who reduces with whom.

Mirrors the reference's `World(swarm)`: ranks from the torchrun environment, stage of a rank
= rank % num_stages (src/world.py:96-97), DP group of a stage = all ranks of that stage, and
the gloo groups the reference creates (src/world.py:32-40). The outer step's collective does
not use those gloo groups: TrainingComm builds an RCCL group over the same ranks.
`World.from_default_group(num_stages)` wraps an already-initialised default process group
(tests, benches) instead of creating the reference's TCPStore.
"""
from __future__ import annotations

import os
from collections import defaultdict
from typing import Dict, List

import torch.distributed as dist


class World:
    def __init__(self, swarm, _init: bool = True):
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.rank = int(os.environ["RANK"]) if _init else dist.get_rank()
        self.local_world_size = int(os.environ.get("LOCAL_WORLD_SIZE", "1"))
        self.world_size = int(os.environ["WORLD_SIZE"]) if _init else dist.get_world_size()
        self.master_addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
        self.master_port = int(os.environ.get("MASTER_PORT", "29500"))
        self.num_stages = swarm.num_stages
        if self.world_size < self.num_stages:
            raise ValueError("World size must be at least num stages")
        self.ranks2stage: Dict[int, int] = defaultdict(
            lambda: -1, {r: r % self.num_stages for r in range(self.world_size)})
        self.stage2ranks: Dict[int, List[int]] = defaultdict(list)
        for r in range(self.world_size):
            self.stage2ranks[self.ranks2stage[r]].append(r)
        self.stage2leader = defaultdict(lambda: -1,
                                        {s: self.stage2ranks[s][0] for s in range(self.num_stages)})
        self.stage = self.ranks2stage[self.rank]
        self.is_first_stage = self.stage == 0
        self.is_last_stage = self.stage == self.num_stages - 1
        self.is_leader = self.rank == self.stage2leader[self.stage]
        self.is_master = self.is_leader and self.is_last_stage
        if _init:
            self.store = dist.TCPStore(host_name=self.master_addr, port=self.master_port + 1,
                                       world_size=self.world_size, is_master=(self.rank == 0))
            dist.init_process_group(backend="gloo", store=self.store, rank=self.rank,
                                    world_size=self.world_size)
        else:
            self.store = None
        # the reference's groups are gloo (its default group is, src/world.py:32-40); say so
        # explicitly, so that a default RCCL group (benches) still gets host-side gloo groups
        # for the p2p headers (any-source receives) and sync_outputs' object all-gather
        pairs = {(s, s + 1): dist.new_group(self.stage2ranks[s] + self.stage2ranks[s + 1],
                                            backend="gloo")
                 for s in range(self.num_stages - 1)}
        self.local_pg = pairs
        self.prev_stage_group = pairs.get((self.stage - 1, self.stage))
        self.next_stage_group = pairs.get((self.stage, self.stage + 1))
        self.curr_stage_group = dist.new_group(self.stage2ranks[self.stage], backend="gloo",
                                               use_local_synchronization=True)
        fl = sorted(set(self.stage2ranks[0] + self.stage2ranks[self.num_stages - 1]))
        self.first_last_stage_group = dist.new_group(fl, backend="gloo",
                                                     use_local_synchronization=True)
        dist.barrier()

    @classmethod
    def from_default_group(cls, num_stages: int = 1) -> "World":
        class _S:
            pass

        s = _S()
        s.num_stages = num_stages
        return cls(s, _init=False)

    @property
    def has_next_stage(self) -> bool:
        return self.stage2ranks[self.stage + 1] != []

    @property
    def has_prev_stage(self) -> bool:
        return self.stage2ranks[self.stage - 1] != []

    @property
    def first_stage_ranks(self) -> List[int]:
        return self.stage2ranks[0]

    @property
    def dp_ranks(self) -> List[int]:
        """Ranks that average pseudo-gradients with this one (src/comm.py:118,122)."""
        return self.stage2ranks[self.stage]
