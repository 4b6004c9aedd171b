"""Multi-GPU = independent replicas.

Boards never interact, so N GPUs run N independent batches with no data-path collective.
One process per GPU (torch.distributed.run sets RANK / LOCAL_RANK / WORLD_SIZE); gloo is
used only for the barrier around the timed region and to combine scalar results (max of
the per-rank times, sum of the per-rank step counts).
"""
import os

SEED_STRIDE_BITS = 40  # rank r draws its Philox stream under key seed + (r << 40)


class Replicas:
    def __init__(self, world_size=None, rank=None, local_rank=None):
        self.world_size = int(os.environ.get("WORLD_SIZE", "1")) if world_size is None else world_size
        self.rank = int(os.environ.get("RANK", "0")) if rank is None else rank
        self.local_rank = int(os.environ.get("LOCAL_RANK", str(self.rank))) if local_rank is None else local_rank
        self._dist = None

    def init(self):
        if self.world_size > 1:
            import torch.distributed as dist

            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if not dist.is_initialized():
                dist.init_process_group("gloo", rank=self.rank, world_size=self.world_size)
            self._dist = dist
        return self

    def board_seed(self, base_seed):
        """Distinct policy stream per rank (same board index on two GPUs plays differently)."""
        return (int(base_seed) + (self.rank << SEED_STRIDE_BITS)) & 0xFFFFFFFFFFFFFFFF

    def global_board_range(self, boards_per_rank):
        """[begin, end) of this rank's boards in the global batch (weak scaling)."""
        return self.rank * boards_per_rank, (self.rank + 1) * boards_per_rank

    def barrier(self):
        if self._dist is not None:
            self._dist.barrier()

    def _reduce(self, x, op):
        if self._dist is None:
            return float(x)
        import torch

        t = torch.tensor([float(x)], dtype=torch.float64)
        self._dist.all_reduce(t, op=op)
        return float(t.item())

    def max(self, x):
        return self._reduce(x, None if self._dist is None else self._dist.ReduceOp.MAX)

    def sum(self, x):
        return self._reduce(x, None if self._dist is None else self._dist.ReduceOp.SUM)

    def close(self):
        if self._dist is not None and self._dist.is_initialized():
            self._dist.destroy_process_group()
        self._dist = None
