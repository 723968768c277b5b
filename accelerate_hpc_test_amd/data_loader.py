"""Data-loading layer: per-rank sharding of samplers/datasets and device-prefetching loaders.

Parity: `/root/reference/src/accelerate/data_loader.py:73-1451` — `SeedableRandomSampler`,
`BatchSamplerShard` (split / no-split, `even_batches` wrap-around), `IterableDatasetShard`,
`DataLoaderShard` (one-batch look-ahead for end-of-data detection), `DataLoaderDispatcher` (rank 0 reads
and broadcasts), `prepare_data_loader`, `skip_first_batches`. The index sequences produced for each rank
are identical to the reference's (tests/test_data_loader.py pins them).

MI355X-native difference: on a GPU, `DataLoaderShard` moves batches with a **device prefetcher**
(`DevicePrefetcher`): a host thread collates the next K batches into pinned memory and issues
`hipMemcpyAsync` (non-blocking `.to`) on a dedicated copy stream, recording a HIP event per batch; the
consumer's compute stream waits on that event instead of the host blocking, so the H2D copy of batch i+1
overlaps compute on batch i. (The reference copies synchronously on the compute stream.)
"""

from __future__ import annotations

import math
import queue
import threading
from contextlib import suppress
from typing import Callable, Optional, Union

import torch
from torch.utils.data import BatchSampler, DataLoader, IterableDataset, RandomSampler

from .logging import get_logger
from .state import DistributedType, GradientState, PartialState
from .utils.dataclasses import RNGType
from .utils.operations import (
    broadcast,
    broadcast_object_list,
    concatenate,
    find_batch_size,
    get_data_structure,
    initialize_tensors,
    send_to_device,
    slice_tensors,
)
from .utils.random import synchronize_rng_states


logger = get_logger(__name__)

# kwargs of the PyTorch DataLoader and their defaults (used to rebuild a user's DataLoader).
_PYTORCH_DATALOADER_KWARGS = {
    "batch_size": 1,
    "shuffle": False,
    "sampler": None,
    "batch_sampler": None,
    "num_workers": 0,
    "collate_fn": None,
    "pin_memory": False,
    "drop_last": False,
    "timeout": 0,
    "worker_init_fn": None,
    "multiprocessing_context": None,
    "generator": None,
    "prefetch_factor": None,
    "persistent_workers": False,
    "pin_memory_device": "",
    "in_order": True,
}


class SeedableRandomSampler(RandomSampler):
    """RandomSampler whose permutation is a function of (`initial_seed` + epoch) — identical on all ranks."""

    def __init__(self, *args, **kwargs):
        data_seed = kwargs.pop("data_seed", None)
        super().__init__(*args, **kwargs)
        self.initial_seed = data_seed if data_seed is not None else torch.random.initial_seed()
        self.epoch = 0

    def __iter__(self):
        if self.generator is None:
            self.generator = torch.Generator()
        self.generator.manual_seed(self.epoch + self.initial_seed)
        yield from super().__iter__()
        self.set_epoch(self.epoch + 1)

    def set_epoch(self, epoch: int):
        self.epoch = epoch


def _check_divisible(who: str, batch_size, num_processes: int):
    """split_batches cuts every batch into num_processes equal slices, so the batch size must divide evenly."""
    if batch_size is None or batch_size % num_processes:
        raise ValueError(f"{who}: split_batches=True cuts each batch into {num_processes} equal slices, which a "
                         f"batch size of {batch_size} does not allow")


class BatchSamplerShard(BatchSampler):
    """Yield only this process's batches of a wrapped `BatchSampler`.

    * `split_batches=False`: process p gets batches p, p+W, p+2W, ...
    * `split_batches=True`: every batch is cut in W equal slices; process p gets slice p.
    With `even_batches=True` the last incomplete round is completed with indices taken cyclically from the
    start of the data so that every process sees the same number of same-sized batches.
    """

    def __init__(self, batch_sampler: BatchSampler, num_processes: int = 1, process_index: int = 0,
                 split_batches: bool = False, even_batches: bool = True):
        bs = getattr(batch_sampler, "batch_size", None)
        if split_batches:
            _check_divisible("BatchSamplerShard", bs, num_processes)
        if bs is None and even_batches:
            raise ValueError("BatchSamplerShard: a batch sampler without a fixed batch_size can only be sharded with "
                             "even_batches=False (Accelerator(even_batches=False) when prepared by the Accelerator)")
        self.batch_sampler, self.batch_size = batch_sampler, bs
        self.num_processes, self.process_index = num_processes, process_index
        self.split_batches, self.even_batches = split_batches, even_batches
        self.drop_last = getattr(batch_sampler, "drop_last", False)

    @property
    def total_length(self):
        return len(self.batch_sampler)

    def __len__(self):
        n = len(self.batch_sampler)
        if self.split_batches:
            return n
        full_rounds, leftover = divmod(n, self.num_processes)
        if leftover == 0 or self.drop_last:
            return full_rounds
        if self.even_batches:
            return full_rounds + 1
        return full_rounds + (1 if self.process_index < leftover else 0)

    def __iter__(self):
        return self._iter_with_split() if self.split_batches else self._iter_with_no_split()

    def _iter_with_split(self):
        bs, W, p = self.batch_size, self.num_processes, self.process_index
        width = bs // W
        first, last = None, None
        for batch in self.batch_sampler:
            if first is None:
                first = list(batch)
            if len(batch) == bs:
                yield batch[width * p : width * (p + 1)]
            last = batch
        if self.drop_last or not first or last is None or len(last) >= bs:
            return
        if not self.even_batches:
            if len(last) > width * p:
                yield last[width * p : width * (p + 1)]
            return
        pool = list(first)
        while len(pool) < bs:
            pool = pool + pool
        completed = list(last) + pool
        yield completed[width * p : width * (p + 1)]

    def _iter_with_no_split(self):
        bs, W, p = self.batch_size, self.num_processes, self.process_index
        round_, pool = [], []
        for idx, batch in enumerate(self.batch_sampler):
            if not self.drop_last and idx < W:
                pool.extend(batch)
            round_.append(batch)
            if len(round_) == W and (bs is None or len(batch) == bs):
                yield round_[p]
                round_ = []
        if self.drop_last or not pool or not round_:
            return
        if not self.even_batches:
            if p < len(round_):
                yield round_[p]
            return
        # Even batches: full batches of the last round go out as they are; the remaining slots of the round
        # (the partial last batch, then any missing batches) are filled cyclically from the start of the data.
        if p < len(round_) and len(round_[p]) == bs:
            yield round_[p]
        while len(pool) < W * bs:
            pool = pool + pool
        last = round_[-1]
        if len(last) < bs:
            slot, carry = len(round_) - 1, list(last)
        else:
            slot, carry = len(round_), []
        cursor = 0
        while slot < W:
            need = bs - len(carry)
            filled = carry + pool[cursor : cursor + need]
            cursor += need
            if slot == p:
                yield filled
            carry = []
            slot += 1


class IterableDatasetShard(IterableDataset):
    """Shard an iterable dataset: consume `W*batch_size` elements, give this process its contiguous slice."""

    def __init__(
        self,
        dataset: IterableDataset,
        batch_size: int = 1,
        drop_last: bool = False,
        num_processes: int = 1,
        process_index: int = 0,
        split_batches: bool = False,
    ):
        if split_batches and batch_size > 1:
            _check_divisible("IterableDatasetShard", batch_size, num_processes)
        self.dataset = dataset
        self.batch_size = batch_size
        self.drop_last = drop_last
        self.num_processes = num_processes
        self.process_index = process_index
        self.split_batches = split_batches

    def set_epoch(self, epoch):
        self.epoch = epoch
        if hasattr(self.dataset, "set_epoch"):
            self.dataset.set_epoch(epoch)

    def __len__(self):
        if self.drop_last:
            return (len(self.dataset) // (self.batch_size * self.num_processes)) * self.batch_size
        return math.ceil(len(self.dataset) / (self.batch_size * self.num_processes)) * self.batch_size

    def __iter__(self):
        if (
            not hasattr(self.dataset, "set_epoch")
            and hasattr(self.dataset, "generator")
            and isinstance(self.dataset.generator, torch.Generator)
        ):
            self.dataset.generator.manual_seed(getattr(self, "epoch", 0))
        global_bs = self.batch_size if self.split_batches else self.batch_size * self.num_processes
        local_bs = self.batch_size // self.num_processes if self.split_batches else self.batch_size
        lo, hi = self.process_index * local_bs, (self.process_index + 1) * local_bs
        first, buf = None, []
        for element in self.dataset:
            buf.append(element)
            if len(buf) == global_bs:
                yield from buf[lo:hi]
                if first is None:
                    first = list(buf)
                buf = []
        if not self.drop_last and buf:
            if first is None:
                first = list(buf)
            while len(buf) < global_bs:
                buf = buf + first
            yield from buf[lo:hi]


class DataLoaderStateMixin:
    """End-of-dataloader / remainder tracking shared with `GradientState`."""

    def __init_subclass__(cls, **kwargs):
        cls.end_of_dataloader = False
        cls.remainder = -1

    def reset(self):
        self.end_of_dataloader = False
        self.remainder = -1

    def begin(self):
        self.reset()
        with suppress(Exception):
            if not self._drop_last:
                length = getattr(self.dataset, "total_dataset_length", len(self.dataset))
                self.remainder = length % self.total_batch_size
        self.gradient_state._add_dataloader(self)

    def end(self):
        self.gradient_state._remove_dataloader(self)


class DevicePrefetcher:
    """Background H2D prefetch of a batch iterator onto a dedicated HIP copy stream.

    A daemon thread pulls CPU batches, pins them, launches non-blocking copies on `copy_stream` and records an
    event; `__next__` makes the *current* stream wait on that event (no host sync) and marks each tensor as used
    by the current stream (`record_stream`) so the caching allocator never recycles it early.

    A consumer that stops early (`break`, an exception, a partially consumed iterator) must not strand the worker in
    a blocking `queue.put` holding `depth` staged device batches: `close()` (called by `DataLoaderShard` when its
    iterator is closed or collected, and by `__del__`) sets a stop flag the worker polls between bounded puts, drains
    the queue and joins the thread.
    """

    _SENTINEL = object()

    def __init__(self, iterator, device: torch.device, depth: int = 2):
        self.iterator = iterator
        device = torch.device(device)
        if device.index is None:
            device = torch.device(device.type, torch.cuda.current_device())
        self.device = device
        self.depth = max(1, depth)
        self.copy_stream = torch.cuda.Stream(device=device, priority=-1)
        self.queue: queue.Queue = queue.Queue(maxsize=self.depth)
        self.error: Optional[BaseException] = None
        self._stop = threading.Event()
        self.thread = threading.Thread(target=self._worker, daemon=True)
        self.thread.start()

    def _put(self, item) -> bool:
        """Bounded put that gives up once the consumer has closed the prefetcher."""
        while not self._stop.is_set():
            try:
                self.queue.put(item, timeout=0.05)
                return True
            except queue.Full:
                continue
        return False

    def close(self, timeout: float = 5.0):
        if self._stop.is_set():
            return
        self._stop.set()
        while True:  # release staged batches (and unblock a worker waiting on a full queue)
            try:
                self.queue.get_nowait()
            except queue.Empty:
                break
        if self.thread.is_alive() and threading.current_thread() is not self.thread:
            self.thread.join(timeout)

    def __del__(self):
        try:
            self.close(timeout=0.5)
        except Exception:
            pass

    def _pin(self, batch):
        def _p(t):
            return t if t.is_pinned() else t.pin_memory()

        from .utils.operations import recursively_apply

        return recursively_apply(_p, batch)

    def _worker(self):
        try:
            torch.cuda.set_device(self.device)
            for batch in self.iterator:
                if self._stop.is_set():
                    return
                with torch.cuda.stream(self.copy_stream):
                    try:
                        staged = send_to_device(self._pin(batch), self.device, non_blocking=True)
                    except RuntimeError:
                        staged = send_to_device(batch, self.device, non_blocking=True)
                    event = torch.cuda.Event()
                    event.record(self.copy_stream)
                if not self._put((staged, event)):
                    return
        except BaseException as e:  # surfaced on the consumer thread
            self.error = e
        self._put(self._SENTINEL)

    def __iter__(self):
        return self

    def __next__(self):
        item = self.queue.get()
        if item is self._SENTINEL:
            if self.error is not None:
                raise self.error
            raise StopIteration
        batch, event = item
        cur = torch.cuda.current_stream(self.device)
        cur.wait_event(event)

        def _rec(t):
            if t.is_cuda:
                t.record_stream(cur)
            return t

        from .utils.operations import recursively_apply

        return recursively_apply(_rec, batch)


class DataLoaderShard(DataLoaderStateMixin, DataLoader):
    """A DataLoader that yields this process's batches, placed on `device`, with one-batch look-ahead so the
    last batch is flagged (`end_of_dataloader`) before it is yielded (needed by gradient accumulation)."""

    def __init__(
        self,
        dataset,
        device=None,
        rng_types=None,
        synchronized_generator=None,
        skip_batches=0,
        use_stateful_dataloader=False,
        _drop_last: bool = False,
        _non_blocking: bool = False,
        torch_device_mesh=None,
        prefetch_to_device: int = 2,
        **kwargs,
    ):
        super().__init__(dataset, **kwargs)
        self.device = device
        self.rng_types = rng_types
        self.synchronized_generator = synchronized_generator
        self.skip_batches = skip_batches
        self.gradient_state = GradientState()
        self._drop_last = _drop_last
        self._non_blocking = _non_blocking
        self.iteration = 0
        self.prefetch_to_device = prefetch_to_device
        self.use_stateful_dataloader = use_stateful_dataloader
        self._batches_yielded = 0
        self._resume_skip = 0

    def _device_iter(self, base_iter):
        dev = self.device
        if dev is not None and torch.device(dev).type == "cuda" and self.prefetch_to_device > 0:
            return DevicePrefetcher(base_iter, torch.device(dev), self.prefetch_to_device)
        if dev is not None:
            return (send_to_device(b, dev, non_blocking=self._non_blocking) for b in base_iter)
        return base_iter

    def __iter__(self):
        if self.rng_types is not None:
            synchronize_rng_states(self.rng_types, self.synchronized_generator)
        self.begin()
        self.set_epoch(self.iteration)
        skip = self.skip_batches + self._resume_skip
        self._resume_skip = 0
        base = super().__iter__()
        # Skipped batches (resume / skip_batches) are drawn from the host iterator before the device prefetcher
        # starts, so none of them is pinned or copied to HBM only to be discarded.
        skipped = 0
        for _ in range(skip):
            try:
                next(base)
            except StopIteration:
                break
            skipped += 1
        it = self._device_iter(base)
        try:
            try:
                current = next(it)
            except StopIteration:
                if skipped:  # the whole epoch was skipped: it still counts as finished
                    self.iteration += 1
                    self._batches_yielded = 0
                self.end()
                return
            index = skipped
            self._batches_yielded = skipped
            while True:
                try:
                    nxt = next(it)
                except StopIteration:
                    self.end_of_dataloader = True
                    self._batches_yielded = index + 1
                    yield current
                    break
                self._batches_yielded = index + 1
                yield current
                index += 1
                current = nxt
            self.iteration += 1
            self._batches_yielded = 0  # a finished epoch resumes at the start of the next one
            self.end()
        finally:  # also on early exit (break / exception / generator collected): stop the prefetch worker
            if isinstance(it, DevicePrefetcher):
                it.close()

    def __reduce__(self):
        args = super().__reduce__()
        return (DataLoaderShard, *args[1:])

    def set_epoch(self, epoch: int):
        if self.iteration != epoch:
            self.iteration = epoch
        if hasattr(self.batch_sampler, "sampler") and hasattr(self.batch_sampler.sampler, "set_epoch"):
            self.batch_sampler.sampler.set_epoch(epoch)
        elif hasattr(self.batch_sampler, "batch_sampler") and hasattr(
            getattr(self.batch_sampler.batch_sampler, "sampler", None), "set_epoch"
        ):
            self.batch_sampler.batch_sampler.sampler.set_epoch(epoch)
        elif hasattr(self.dataset, "set_epoch"):
            self.dataset.set_epoch(epoch)

    @property
    def total_batch_size(self):
        batch_sampler = self.sampler if isinstance(self.sampler, BatchSampler) else self.batch_sampler
        return (
            batch_sampler.batch_size
            if getattr(batch_sampler, "split_batches", False)
            else (batch_sampler.batch_size * getattr(batch_sampler, "num_processes", 1))
        )

    @property
    def total_dataset_length(self):
        if hasattr(self.dataset, "total_length"):
            return self.dataset.total_length
        return len(self.dataset)

    def get_sampler(self):
        return get_sampler(self)

    def set_sampler(self, sampler):
        sampler_is_batch_sampler = isinstance(self.sampler, BatchSampler)
        if sampler_is_batch_sampler:
            self.sampler.sampler = sampler
        else:
            self.batch_sampler.sampler = sampler
            if hasattr(self.batch_sampler, "batch_sampler"):
                self.batch_sampler.batch_sampler.sampler = sampler

    # Native resumable state (position within the epoch); replaces torchdata's StatefulDataLoader.
    def state_dict(self):
        return {"iteration": self.iteration, "batches_yielded": self._batches_yielded}

    def load_state_dict(self, state_dict):
        self.iteration = state_dict.get("iteration", 0)
        self._resume_skip = state_dict.get("batches_yielded", 0)


def _shuffling_datapipe(dataset) -> bool:
    try:
        from torch.utils.data.datapipes.iter.combinatorics import ShufflerIterDataPipe
    except ImportError:
        return False
    return isinstance(dataset, ShufflerIterDataPipe) and bool(dataset._shuffle_enabled)


class DataLoaderDispatcher(DataLoaderStateMixin, DataLoader):
    """Rank 0 iterates the underlying loader and broadcasts each (concatenated or split) batch; every rank
    keeps its slice. One object broadcast (structure) + one coalesced tensor broadcast per step."""

    def __init__(self, dataset, split_batches: bool = False, skip_batches=0, use_stateful_dataloader=False,
                 _drop_last: bool = False, _non_blocking: bool = False, slice_fn=None, torch_device_mesh=None,
                 **kwargs):
        reshuffle = _shuffling_datapipe(dataset)  # DataLoader.__init__ resets a shuffler datapipe's switch
        super().__init__(dataset, **kwargs)
        if reshuffle:
            torch.utils.data.graph_settings.apply_shuffle_settings(dataset, shuffle=True)
        self.state, self.gradient_state = PartialState(), GradientState()
        self.split_batches, self.skip_batches = split_batches, skip_batches
        self._drop_last, self._non_blocking = _drop_last, _non_blocking
        self.slice_fn = slice_fn or slice_tensors
        self.torch_device_mesh = torch_device_mesh
        self.use_stateful_dataloader = use_stateful_dataloader
        self.iteration = self._batches_yielded = self._resume_skip = 0

    _MIXED_SIZES = ("You can't use batches of different size with `dispatch_batches=True` or when using an `IterableDataset`. "
                    "Either pass `dispatch_batches=False` and have each process fetch its own batch or pass "
                    "`split_batches=True`.")

    def _rank0_next(self, it):
        """Rank 0: the next GLOBAL batch — one loader batch (split_batches), else `num_processes` loader batches
        concatenated; a short final group is kept unless drop_last. None at the end."""
        if self.split_batches:
            return next(it, None)
        group = []
        for _ in range(self.state.num_processes):
            b = next(it, None)
            if b is None:
                break
            group.append(b)
        if not group or (len(group) < self.state.num_processes and self._drop_last):
            return None
        try:
            return concatenate(group, dim=0)
        except RuntimeError as exc:
            raise RuntimeError(self._MIXED_SIZES) from exc

    def _next_global(self, it):
        """Every rank: the next global batch on this device (rank 0's, broadcast: its structure as one object, then
        its tensors), or None at the end."""
        batch = self._rank0_next(it) if self.state.process_index == 0 else None
        info = [get_data_structure(batch) if batch is not None else None]
        broadcast_object_list(info)
        if info[0] is None:
            return None
        if self.state.process_index != 0:
            batch = initialize_tensors(info[0])
        batch = send_to_device(batch, self.state.device, non_blocking=self._non_blocking)
        return broadcast(batch, from_process=0)

    def __iter__(self):
        self.begin()
        self.set_epoch(self.iteration)
        P, r = self.state.num_processes, self.state.process_index
        skip = self.skip_batches + self._resume_skip  # a restored position applies to this pass only
        self._resume_skip = 0
        it = super().__iter__() if r == 0 else None
        head = None  # first P samples of the epoch: pad a final global batch that does not split evenly
        cur, index = self._next_global(it), 0
        while cur is not None:
            nxt = self._next_global(it)  # one batch of look-ahead: the last batch is known when it is handed out
            last = nxt is None
            if not self._drop_last and head is None:
                head = self.slice_fn(cur, slice(0, P), process_index=r, num_processes=P)
            seen = find_batch_size(cur)
            per = seen // P
            if last and not self._drop_last and seen % P != 0:
                cur = concatenate([cur, head], dim=0)
                per += 1
            mine = self.slice_fn(cur, slice(r * per, (r + 1) * per), process_index=r, num_processes=P)
            if last:
                self.end_of_dataloader = True
                self.remainder = seen
            if index >= skip:
                self._batches_yielded = index + 1
                yield mine
            index += 1
            cur = nxt
        self.iteration += 1
        self._batches_yielded = 0
        self.end()

    def set_epoch(self, epoch: int):
        if self.iteration != epoch:
            self.iteration = epoch
        if hasattr(self.batch_sampler, "sampler") and hasattr(self.batch_sampler.sampler, "set_epoch"):
            self.batch_sampler.sampler.set_epoch(epoch)
        elif hasattr(self.dataset, "set_epoch"):
            self.dataset.set_epoch(epoch)

    def __len__(self):
        whole_length = super().__len__()
        if self.split_batches:
            return whole_length
        elif self._drop_last:
            return whole_length // self.state.num_processes
        return math.ceil(whole_length / self.state.num_processes)

    def __reduce__(self):
        args = super().__reduce__()
        return (DataLoaderDispatcher, *args[1:])

    @property
    def total_batch_size(self):
        return self.dataset.batch_size if self.split_batches else (self.dataset.batch_size * self.dataset.num_processes)

    @property
    def total_dataset_length(self):
        return len(self.dataset)

    def get_sampler(self):
        return get_sampler(self)

    def set_sampler(self, sampler):
        sampler_is_batch_sampler = isinstance(self.sampler, BatchSampler)
        if sampler_is_batch_sampler:
            self.sampler.sampler = sampler
        else:
            self.batch_sampler.sampler = sampler
            if hasattr(self.batch_sampler, "batch_sampler"):
                self.batch_sampler.batch_sampler.sampler = sampler

    def state_dict(self):
        return {"iteration": self.iteration, "batches_yielded": self._batches_yielded}

    def load_state_dict(self, state_dict):
        self.iteration = state_dict.get("iteration", 0)
        self._resume_skip = state_dict.get("batches_yielded", 0)


def get_sampler(dataloader):
    """The sampler of a dataloader, looking through a BatchSampler used as sampler."""
    sampler_is_batch_sampler = isinstance(dataloader.sampler, BatchSampler)
    if sampler_is_batch_sampler:
        sampler = getattr(dataloader.sampler, "sampler", None)
    else:
        sampler = getattr(dataloader.batch_sampler, "sampler", None)
    return sampler


def _maybe_seedable(sampler, use_seedable_sampler: bool, data_seed):
    """A RandomSampler becomes a SeedableRandomSampler (epoch-seeded, identical on every rank) when requested."""
    if isinstance(sampler, RandomSampler) and use_seedable_sampler:
        return SeedableRandomSampler(data_source=sampler.data_source, replacement=sampler.replacement,
                                     num_samples=sampler._num_samples,
                                     generator=getattr(sampler, "generator", None) or torch.Generator(), data_seed=data_seed)
    return sampler


class _ShardPlan:
    """What this rank iterates: the (possibly wrapped) dataset, the (possibly sharded) batch sampler, and the generator
    every rank must keep in lock-step so shuffles agree."""

    def __init__(self, dataset, batch_sampler, generator, sampler_is_batch_sampler):
        self.dataset, self.batch_sampler = dataset, batch_sampler
        self.generator, self.sampler_is_batch_sampler = generator, sampler_is_batch_sampler

    @classmethod
    def build(cls, dl, sampler, num_processes, process_index, split_batches, even_batches, dispatch_batches,
              use_seedable_sampler):
        iterable = isinstance(dl.dataset, IterableDataset)
        as_batch_sampler = isinstance(dl.sampler, BatchSampler)
        plan = cls(dl.dataset, None if iterable else dl.batch_sampler, None, as_batch_sampler)
        if num_processes == 1 or dispatch_batches:
            return plan  # one process, or rank 0 reads everything and dispatches
        if iterable:
            plan.generator = getattr(dl.dataset, "generator", None)
            plan.dataset = IterableDatasetShard(dl.dataset, batch_size=dl.batch_size, drop_last=dl.drop_last,
                                                num_processes=num_processes, process_index=process_index,
                                                split_batches=split_batches)
            return plan
        if not use_seedable_sampler and hasattr(sampler, "generator"):
            if sampler.generator is None:  # give the shuffle a generator every rank can seed identically
                sampler.generator = torch.Generator()
                sampler.generator.manual_seed(int(torch.empty((), dtype=torch.int64).random_().item()))
            plan.generator = sampler.generator
        plan.batch_sampler = BatchSamplerShard(dl.sampler if as_batch_sampler else dl.batch_sampler,
                                               num_processes=num_processes, process_index=process_index,
                                               split_batches=split_batches, even_batches=even_batches)
        return plan


def _rebuild_kwargs(dl, shard: "_ShardPlan", num_processes, split_batches, dispatch_batches) -> dict:
    """The original loader's DataLoader arguments minus the ones the shard plan replaces; loaders without a batch
    sampler (iterable datasets) keep batch_size / drop_last (per-process batch size with split_batches)."""
    replaced = {"batch_size", "shuffle", "sampler", "batch_sampler", "drop_last"}
    kw = {k: getattr(dl, k, default) for k, default in _PYTORCH_DATALOADER_KWARGS.items() if k not in replaced and hasattr(dl, k)}
    if shard.batch_sampler is None:
        kw["drop_last"] = dl.drop_last
        kw["batch_size"] = dl.batch_size // num_processes if split_batches and not dispatch_batches else dl.batch_size
    return kw


def prepare_data_loader(
    dataloader: DataLoader,
    device: Optional[torch.device] = None,
    num_processes: Optional[int] = None,
    process_index: Optional[int] = None,
    split_batches: bool = False,
    put_on_device: bool = False,
    rng_types: Optional[list[Union[str, RNGType]]] = None,
    dispatch_batches: Optional[bool] = None,
    even_batches: bool = True,
    slice_fn_for_dispatch: Optional[Callable] = None,
    use_seedable_sampler: bool = False,
    data_seed: Optional[int] = None,
    non_blocking: bool = False,
    use_stateful_dataloader: bool = False,
    torch_device_mesh=None,
    prefetch_to_device: int = 2,
) -> DataLoader:
    """Rebuild `dataloader` so it yields only this process's share (reference `data_loader.py:996-1309`)."""
    if dispatch_batches is None:
        dispatch_batches = False if not put_on_device else isinstance(dataloader.dataset, IterableDataset)
    if dispatch_batches and not put_on_device:
        raise ValueError("Using `dispatch_batches=True` requires `put_on_device=True`.")
    state = PartialState()
    if num_processes is None:
        num_processes = state.num_processes
    if process_index is None:
        process_index = state.process_index

    # With a device mesh, ranks that share a TP/CP/SP group must see the same data: remap to data-parallel
    # coordinates (reference `data_loader.py:1109-1145`).
    if torch_device_mesh is not None:
        dp_size, dp_rank = torch_device_mesh.data_parallel_size_and_rank()
        num_processes, process_index = dp_size, dp_rank

    if split_batches:
        if dataloader.batch_size is not None:
            batch_size_for_check = dataloader.batch_size
        else:
            batch_size_for_check = getattr(dataloader.batch_sampler, "batch_size", None)
        if batch_size_for_check is not None and batch_size_for_check > 1 and batch_size_for_check % num_processes != 0:
            raise ValueError(
                f"To use a `DataLoader` in `split_batches` mode, the batch size ({dataloader.batch_size}) "
                f"needs to be a round multiple of the number of processes ({num_processes})."
            )

    sampler = _maybe_seedable(get_sampler(dataloader), use_seedable_sampler, data_seed)
    shard = _ShardPlan.build(dataloader, sampler, num_processes, process_index, split_batches, even_batches,
                             dispatch_batches, use_seedable_sampler)
    if rng_types is not None and shard.generator is None:
        rng_types = [r for r in rng_types if r != "generator"]  # nothing to synchronise
    kwargs = _rebuild_kwargs(dataloader, shard, num_processes, split_batches, dispatch_batches)
    common = {"_drop_last": dataloader.drop_last, "_non_blocking": non_blocking,
              "use_stateful_dataloader": use_stateful_dataloader}
    if dispatch_batches:
        kwargs.pop("generator", None)  # only rank 0 draws samples
        dataloader = DataLoaderDispatcher(shard.dataset, split_batches=split_batches, batch_sampler=shard.batch_sampler,
                                          slice_fn=slice_fn_for_dispatch, torch_device_mesh=torch_device_mesh, **common,
                                          **kwargs)
    else:
        shard_kw = {"device": device if put_on_device else None, "rng_types": rng_types,
                    "synchronized_generator": shard.generator, "prefetch_to_device": prefetch_to_device}
        if shard.sampler_is_batch_sampler:  # a BatchSampler passed as `sampler` stays in that slot
            dataloader = DataLoaderShard(shard.dataset, sampler=shard.batch_sampler, batch_size=dataloader.batch_size,
                                         **shard_kw, **common, **kwargs)
        else:
            dataloader = DataLoaderShard(shard.dataset, batch_sampler=shard.batch_sampler, **shard_kw, **common, **kwargs)
    if isinstance(sampler, SeedableRandomSampler) and use_seedable_sampler:
        dataloader.set_sampler(sampler)
    return dataloader


class SkipBatchSampler(BatchSampler):
    """Skip the first `skip_batches` batches of a batch sampler."""

    def __init__(self, batch_sampler, skip_batches=0):
        self.batch_sampler = batch_sampler
        self.skip_batches = skip_batches

    def __iter__(self):
        for index, samples in enumerate(self.batch_sampler):
            if index >= self.skip_batches:
                yield samples

    @property
    def total_length(self):
        return len(self.batch_sampler)

    def __len__(self):
        return len(self.batch_sampler) - self.skip_batches


class SkipDataLoader(DataLoaderStateMixin, DataLoader):
    """A plain DataLoader that skips its first `skip_batches` batches."""

    def __init__(self, dataset, skip_batches=0, use_stateful_dataloader=False, **kwargs):
        super().__init__(dataset, **kwargs)
        self.skip_batches = skip_batches
        self.gradient_state = GradientState()
        self._drop_last = kwargs.get("drop_last", False)

    def __iter__(self):
        self.begin()
        for index, batch in enumerate(super().__iter__()):
            if index >= self.skip_batches:
                yield batch
        self.end()

    def __len__(self):
        return super().__len__() - self.skip_batches

    @property
    def total_batch_size(self):
        return self.batch_size or 1


_SAMPLING_KWARGS = frozenset({"batch_size", "shuffle", "sampler", "batch_sampler", "drop_last"})


def skip_first_batches(dataloader, num_batches=0):
    """A loader equivalent to `dataloader` that starts after its first `num_batches` batches (mid-epoch resume).

    Map-style data: the (batch) sampler is wrapped in a `SkipBatchSampler`, so skipped batches are never loaded or
    uploaded. Iterable data has no sampler to advance: the new loader drops the first batches it produces."""
    dataset = dataloader.dataset
    kw = {k: getattr(dataloader, k) for k in _PYTORCH_DATALOADER_KWARGS
          if k not in _SAMPLING_KWARGS and hasattr(dataloader, k)}
    if isinstance(dataset, IterableDataset):
        kw.update(batch_size=dataloader.batch_size, drop_last=dataloader.drop_last)
        skipped, sampler_is_batches = None, False
    else:
        sampler_is_batches = isinstance(dataloader.sampler, BatchSampler)
        source = dataloader.sampler if sampler_is_batches else dataloader.batch_sampler
        skipped = SkipBatchSampler(source, skip_batches=num_batches)

    if isinstance(dataloader, DataLoaderDispatcher):
        kw.pop("generator", None)  # rank 0 draws the batches; the dispatcher makes its own generator
        kw.update({"skip_batches": num_batches} if skipped is None else {"batch_sampler": skipped})
        return DataLoaderDispatcher(dataset, split_batches=dataloader.split_batches,
                                    _drop_last=dataloader._drop_last, **kw)
    if isinstance(dataloader, DataLoaderShard):
        if skipped is None:
            kw["skip_batches"] = num_batches
        elif sampler_is_batches:
            kw.update(sampler=skipped, batch_size=dataloader.batch_size)
        else:
            kw["batch_sampler"] = skipped
        return DataLoaderShard(dataset, device=dataloader.device, rng_types=dataloader.rng_types,
                               synchronized_generator=dataloader.synchronized_generator,
                               _drop_last=dataloader._drop_last, prefetch_to_device=dataloader.prefetch_to_device,
                               **kw)
    if skipped is None:
        return SkipDataLoader(dataset, skip_batches=num_batches, **kw)
    return DataLoader(dataset, batch_sampler=skipped, **kw)
