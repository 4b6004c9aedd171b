"""Multi-GPU = independent replicas.

Boards never interact, so N GPUs run N independent batches with no data-path collective;
the only cross-GPU data are a few host-side scalars (steps, nodes, times).  Two ways to get
N replicas, neither needing PyTorch:

* threads (preferred; `bench.py --gpus N` run directly): ONE process, one host thread and
  one gc_env / gc_engine handle per device.  ctypes releases the GIL for every C-ABI call,
  and a whole timed region is a single call per replica (gc_env_step_random launches K
  kernels), so the threads drive their devices concurrently.
* processes (`python -m torch.distributed.run --nproc-per-node N bench.py --gpus N`, the
  launcher the driver uses): one process per GPU, RANK / WORLD_SIZE / LOCAL_RANK from the
  environment.  The barrier and the max / sum of per-rank scalars go through a file group
  in the node's temp directory (all ranks share one node; keyed by the launcher's pid, so
  concurrent launches never meet).  GC_REPLICA_BACKEND=gloo uses torch.distributed's gloo
  instead (the only place torch is ever imported).

Replica r (0 <= r < world_size) owns global boards [r*B, (r+1)*B) and draws its policy
stream under the Philox key seed + (r << 40).
"""
import json
import os
import tempfile
import threading
import time

SEED_STRIDE_BITS = 40  # replica r draws its Philox stream under key seed + (r << 40)


class Replica:
    """One replica: its global index and the device it runs on."""

    def __init__(self, index, device):
        self.index = int(index)
        self.device = int(device)

    def board_seed(self, base_seed):
        """Distinct policy stream per replica (same board index on two GPUs plays differently)."""
        return (int(base_seed) + (self.index << SEED_STRIDE_BITS)) & 0xFFFFFFFFFFFFFFFF

    def board_range(self, boards_per_replica):
        """[begin, end) of this replica's boards in the global batch (weak scaling)."""
        return self.index * boards_per_replica, (self.index + 1) * boards_per_replica


def _remove_stale_groups():
    """A group's files stay until its launcher is gone (a rank cannot know when the others
    have read its last record); groups of launchers that no longer exist are removed here."""
    import glob
    import shutil

    for d in glob.glob(os.path.join(tempfile.gettempdir(), "gymchess_replicas_*")):
        try:
            pid = int(os.path.basename(d).split("_")[2])
            os.kill(pid, 0)
        except (ValueError, IndexError):
            continue
        except ProcessLookupError:
            shutil.rmtree(d, ignore_errors=True)
        except PermissionError:
            continue


class _FileGroup:
    """Barrier + all-gather of small JSON values among the ranks of one node, through one file
    per rank.  A rank's file holds its latest round and the values of its last two rounds: a
    rank can run at most one round ahead of the slowest (it cannot pass round k before every
    rank has reached k), so a reader of round k finds it as `cur` or `prev`."""

    def __init__(self, rank, world, key, timeout=900.0):
        self.rank, self.world, self.timeout = rank, world, timeout
        self.dir = os.path.join(tempfile.gettempdir(), f"gymchess_replicas_{key}")
        _remove_stale_groups()
        os.makedirs(self.dir, exist_ok=True)
        self.round = 0
        self.prev = None

    def _path(self, r):
        return os.path.join(self.dir, f"rank{r}.json")

    def _read(self, r):
        try:
            with open(self._path(r)) as f:
                return json.load(f)
        except (FileNotFoundError, json.JSONDecodeError):
            return None

    def allgather(self, value):
        k = self.round
        self.round += 1
        rec = {"round": k, "cur": value, "prev": self.prev}
        self.prev = value
        tmp = self._path(self.rank) + f".tmp{os.getpid()}"
        with open(tmp, "w") as f:
            json.dump(rec, f)
        os.replace(tmp, self._path(self.rank))  # atomic: readers see the old or the new record
        out = [None] * self.world
        t0 = time.monotonic()
        pending = set(range(self.world))
        while pending:
            for r in list(pending):
                d = self._read(r)
                if d is not None and d["round"] >= k:
                    out[r] = d["cur"] if d["round"] == k else d["prev"]
                    pending.discard(r)
            if pending:
                if time.monotonic() - t0 > self.timeout:
                    raise TimeoutError(f"replica group: ranks {sorted(pending)} never reached round {k}")
                time.sleep(0.0005)
        return out


def overlap(spans):
    """How the timed regions [begin, end) of N replicas overlapped in wall time: union_wall_s
    (first begin to last end), the common interval (last begin to first end) as a fraction of
    the longest region (min_overlap: 1 = all ran over the same interval, 0 = some two never
    overlapped) and the begin skew."""
    spans = [(float(a), float(b)) for a, b in spans]
    if not spans:
        return None
    first, last = min(a for a, _ in spans), max(b for _, b in spans)
    common = min(b for _, b in spans) - max(a for a, _ in spans)
    longest = max(b - a for a, b in spans)
    return {"replicas": len(spans), "union_wall_s": last - first,
            "min_overlap": max(0.0, common) / longest if longest > 0 else 1.0,
            "begin_skew_s": max(a for a, _ in spans) - first, "longest_s": longest}


class Replicas:
    """mode: None = "processes" under a launcher (WORLD_SIZE in the environment or world_size
    given), else "threads"; "threads" forces one process with a thread per device whatever
    the environment says (MultiDeviceChessEnv's device_ids contract inside a launched job)."""

    def __init__(self, gpus=None, world_size=None, rank=None, local_rank=None, devices=None, mode=None):
        if mode not in (None, "threads", "processes"):
            raise ValueError(f"mode must be None, 'threads' or 'processes', not {mode!r}")
        procs = mode == "processes" or (mode is None and ("WORLD_SIZE" in os.environ or world_size is not None))
        if procs:  # one process per GPU
            self.mode = "processes"
            self.world_size = int(os.environ.get("WORLD_SIZE", "1")) if world_size is None else int(world_size)
            self.rank = int(os.environ.get("RANK", "0")) if rank is None else int(rank)
            lr = int(os.environ.get("LOCAL_RANK", str(self.rank)) if local_rank is None else local_rank)
            # devices maps local ranks to devices (default: the local rank; the 1-GPU tests put
            # several ranks on device 0)
            self.local = [Replica(self.rank, lr if devices is None else int(devices[lr]))]
            if gpus is not None and int(gpus) != self.world_size:
                raise ValueError(f"--gpus {gpus} does not match the launcher's WORLD_SIZE={self.world_size}")
        else:  # one process, one thread per device
            self.mode = "threads"
            self.world_size = 1 if gpus is None else int(gpus)
            if self.world_size < 1:
                raise ValueError("--gpus must be >= 1")
            self.rank = 0
            devs = list(range(self.world_size)) if devices is None else [int(d) for d in devices]
            if len(devs) != self.world_size:
                raise ValueError(f"{len(devs)} devices for {self.world_size} replicas")
            # devices may repeat (several replicas on one GPU: the 1-GPU tests of this path)
            self.local = [Replica(r, d) for r, d in enumerate(devs)]
        self._group = None
        self._dist = None
        self.last_overlap = None

    def init(self):
        if self.mode == "processes" and self.world_size > 1:
            if os.environ.get("GC_REPLICA_BACKEND", "file") == "gloo":
                import torch.distributed as dist

                os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
                if not dist.is_initialized():
                    dist.init_process_group("gloo", rank=self.rank, world_size=self.world_size)
                self._dist = dist
            else:
                # the launcher's pid and port, and its restart count: workers restarted by
                # torchrun (--max-restarts) keep pid and port but must not read the previous
                # attempt's records
                key = os.environ.get("GC_REPLICA_KEY") or "_".join(
                    (str(os.getppid()), os.environ.get("MASTER_PORT", "0"),
                     os.environ.get("TORCHELASTIC_RESTART_COUNT", "0"),
                     "".join(c for c in os.environ.get("TORCHELASTIC_RUN_ID", "") if c.isalnum())[:32]))
                self._group = _FileGroup(self.rank, self.world_size, key)
        return self

    # ------------------------------------------------------------------ local replicas
    def run(self, fn):
        """fn(replica) on every local replica, one thread each; results in replica order.
        An exception in any thread is re-raised here."""
        if len(self.local) == 1:
            return [fn(self.local[0])]
        res = [None] * len(self.local)
        err = []

        def body(k, rp):
            try:
                res[k] = fn(rp)
            except BaseException as ex:  # noqa: BLE001 -- re-raised in the caller
                err.append(ex)

        th = [threading.Thread(target=body, args=(k, rp)) for k, rp in enumerate(self.local)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        if err:
            raise err[0]
        return res

    def timed(self, fn):
        """Barrier, then fn(replica) on every local replica started together (a thread
        barrier), each timing itself; returns (results, the max of the replicas' seconds over
        the whole job).  fn returns (result, seconds) or (result, seconds, t_begin) with t_begin
        its region's start by time.perf_counter() -- CLOCK_MONOTONIC, one clock for every
        process of the node -- and then self.last_overlap describes how the regions of all
        replicas of all ranks overlapped (overlap())."""
        gate = threading.Barrier(len(self.local))

        def body(rp):
            gate.wait()
            return fn(rp)

        self.barrier()
        out = self.run(body)
        spans = [(o[2], o[2] + o[1]) for o in out if len(o) > 2]
        # every rank issues the same collective whatever its fn returned (a rank
        # skipping it would leave the others waiting); overlap only when every replica timed one
        got = self.allgather({"spans": spans, "complete": len(spans) == len(out)})
        self.last_overlap = (overlap([tuple(x) for g in got for x in g["spans"]])
                             if all(g["complete"] for g in got) else None)
        return [o[0] for o in out], self.max(max(o[1] for o in out))

    def allgather(self, value):
        """every rank's value (JSON-able), in rank order, concatenated when they are lists"""
        if self._group is not None:
            vals = self._group.allgather(value)
        elif self._dist is not None:
            vals = [None] * self.world_size
            self._dist.all_gather_object(vals, value)
        else:
            vals = [value]
        if all(isinstance(v, list) for v in vals):
            return [x for v in vals for x in v]
        return vals

    # ------------------------------------------------------------------ across processes
    def barrier(self):
        if self._group is not None:
            self._group.allgather(None)
        elif self._dist is not None:
            self._dist.barrier()

    def _reduce(self, x, op):
        if self._group is not None:
            vals = self._group.allgather(float(x))
            return max(vals) if op == "max" else sum(vals)
        if self._dist is not None:
            import torch

            t = torch.tensor([float(x)], dtype=torch.float64)
            self._dist.all_reduce(t, op=self._dist.ReduceOp.MAX if op == "max" else self._dist.ReduceOp.SUM)
            return float(t.item())
        return float(x)

    def max(self, x):
        return self._reduce(x, "max")

    def sum(self, x):
        return self._reduce(x, "sum")

    def close(self):
        if self._group is not None:
            self._group.allgather(None)  # nobody leaves while another rank still reads
        if self._dist is not None and self._dist.is_initialized():
            self._dist.destroy_process_group()
        self._dist = None
