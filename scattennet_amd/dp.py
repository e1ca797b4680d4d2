"""Batch-sharded data parallelism over RCCL.

The reference initialises an NCCL process group but never wraps the model in DDP nor
all-reduces a gradient (utils.py:237-265, main.py:132-133), so this is the
north-star's new functionality: one process per GPU, each running its own clips through the
HIP path, the fp32 gradients averaged over all ranks every step (torch.distributed backend
"nccl" is RCCL on ROCm).

`GradBuckets` is the reducer.  It installs itself as the parameter-gradient sink of
`ops` (ops.param_grad_empty / ops.params_produced):

* Plan.  The first backward runs unbucketed and records the order in which the backward
  produces parameter gradients.  The gradients are then laid out in that order in ONE flat
  fp32 buffer, cut into buckets of about `bucket_mb` MB (default 25: four buckets for the
  103 MB of the 4-stream SCA) — the bucket holding the top layers' gradients fills first.
  Parameters that never receive a gradient (the ResidualNetwork long shortcuts, SURVEY.md
  §7) get no slot and keep `.grad = None`, as in the reference; so do parameters whose
  gradient arrives in more than one piece (autograd would add the pieces outside our
  streams) and parameters produced outside the `ops` sites — those are reduced by a
  fallback all-reduce after the backward.
* Steps.  Every kernel writing a planned gradient writes straight into that parameter's
  slot (no flatten / copy-back), and `.grad` is left as a view of the slot.  With the
  overlapped mode (RCCL), the moment a bucket's last gradient has been enqueued, the
  bucket's all-reduce is issued on a communication stream that waits on exactly the
  streams that produced its gradients (the weight-gradient side streams), so it runs under
  the backward of the layers below; the caller's stream joins the communication stream when
  the backward completes (an autograd final callback).  All of this is capture-safe: the
  bench captures forward + backward + the bucketed all-reduces in one hipGraph.
  Without overlap (the `gloo` rehearsal backend, or SCA_DP_OVERLAP=0), `sync()` after the
  backward (or graph replay) all-reduces the flat buffer in place.
* Averaging: over RCCL one AVG all-reduce per bucket (ncclAvg: the 1/world scale inside the
  collective, no separate scaling kernel over the 100 MB); over gloo (no AVG) the bucket is
  pre-scaled by 1/world, then SUM all-reduced (exact for power-of-two world sizes).
* Streams.  Every collective is issued in torch's synchronous form (`async_op=False`), which
  ProcessGroupNCCL runs on the CURRENT stream (torch >= 2.8; probed on the box by
  tools/dp_capture_diag.py "watchdog_fixed"), from one of two private communication streams:
  one for eager steps, one used only while a hipGraph is being captured.  ProcessGroupNCCL's
  watchdog thread polls the end event of every eager collective until it retires it (every
  100 ms); hipEventQuery on an event whose stream is capturing at that moment fails with
  hipErrorCapturedEvent, and the watchdog then terminates the process.  With the eager and
  the captured collectives on disjoint streams, no event the watchdog can hold is ever on a
  capturing stream, whatever the timing (the round-4 aborts were this race —
  the async form put both on the process group's one internal stream).

Oracle: the averaged all-reduced gradient times the world size equals the single-process
gradient of the whole global batch (sum loss) — tests/test_dp.py checks the reducer with
`gloo`; tests/test_gpu_dp.py checks batch additivity of the HIP gradients and the captured
bucketed path at world size 1 on RCCL.
"""
import os

import torch
import torch.distributed as dist

from . import ops

_ALIGN = 64  # floats: every slot starts on a 256-byte boundary


class GradBuckets:
    def __init__(self, params, world=None, bucket_mb=None, overlap=None, average=True):
        self.params = [p for p in params if p.requires_grad]
        self.world = world if world is not None else (dist.get_world_size() if dist.is_initialized() else 1)
        self.average = average
        self.bucket_bytes = int(float(bucket_mb if bucket_mb is not None else
                                      os.environ.get("SCA_DP_BUCKET_MB", "25")) * 2 ** 20)
        backend = dist.get_backend() if dist.is_initialized() else None
        self.backend = backend  # "nccl" (RCCL): AVG all-reduces; any other: pre-scale + SUM
        if overlap is None:
            overlap = backend == "nccl" and os.environ.get("SCA_DP_OVERLAP", "1") != "0"
        self.overlap = bool(overlap)
        # issue the collectives even at world size 1 (SCA_DP_FORCE=1: rehearse the captured
        # RCCL path on a one-GPU box; the all-reduce is then an identity)
        self.collective = self.world > 1 or (dist.is_initialized() and os.environ.get("SCA_DP_FORCE", "0") != "0")
        self._key = {self._k(p): i for i, p in enumerate(self.params)}
        self.plan = None          # list of buckets: (offset, numel, [param indices])
        self.flat = None
        self.slot = {}            # param index -> (offset, numel)
        self.bucket_of = {}       # param index -> bucket index
        self._order, self._count = [], {}
        self._comms = {}          # False: eager communication stream, True: the capture-only one
        # a completed bucket's all-reduce is forked at the NEXT gradient report (from events
        # recorded when it completed): see produced()
        self.defer = os.environ.get("SCA_DP_DEFER", "1") != "0"
        self._step = None
        self.last_fallback = []   # parameter indices reduced by the fallback in the last step
        ops.set_grad_sink(self)

    # ------------------------------------------------------------------ helpers
    @staticmethod
    def _k(p):
        return (p.data_ptr(), p.numel())

    def _index(self, p):
        return self._key.get(self._k(p))

    def close(self):
        if ops._GRAD_SINK is self:
            ops.set_grad_sink(None)

    def _stream(self):
        return torch.cuda.current_stream() if self.params[0].is_cuda else None

    def _begin(self):
        """First sink call of a backward: choose this step's mode and queue its finish.  A step
        left by a backward that raised before its finish callback is drained first: its issued
        all-reduces (the same on every rank) complete before this step writes the buckets
        again; its not yet issued ones are dropped."""
        stale = self._step
        if stale is not None:
            for work in stale["works"]:
                work.wait()
            cur = self._stream()
            if cur is not None:
                for comm in stale["comms"].values():
                    cur.wait_stream(comm)
                    ops.note_join(cur, comm)
        fast = self.plan is not None and all(self.params[i].grad is None for i in self.slot)
        self._step = {"task": torch._C._current_graph_task_id(),
                      "fast": fast, "pending": [len(b[2]) for b in self.plan] if fast else None,
                      "streams": [dict() for _ in self.plan] if fast else None, "works": [],
                      "seen": set(), "producers": {}, "comms": {}, "ready": []}
        torch.autograd.Variable._execution_engine.queue_callback(self._finish)

    # ------------------------------------------------------------------ sink protocol (ops)
    def _current(self):
        """This backward's step state: begun at its first sink call.  A state left by a backward
        that raised before its finish callback (another autograd graph task) is discarded."""
        if self._step is None or self._step["task"] != torch._C._current_graph_task_id():
            self._begin()
        return self._step

    def grad_buffer(self, p):
        self._current()
        if not self._step["fast"]:
            return None
        i = self._index(p)
        if i is None or i not in self.slot or p.grad is not None:
            return None
        o, n = self.slot[i]
        return self.flat[o:o + n].view(p.shape)

    def produced(self, params):
        st = self._current()
        self._launch_ready()  # buckets completed at the previous report
        stream = self._stream()
        if stream is not None:
            st["producers"][stream.cuda_stream] = stream
        for p in params:
            i = self._index(p)
            if i is None:
                continue
            if self.plan is None:  # discovery step: record the production order
                if i not in self._count:
                    self._order.append(i)
                self._count[i] = self._count.get(i, 0) + 1
                continue
            if not st["fast"] or i not in self.slot or i in st["seen"]:
                continue
            st["seen"].add(i)
            b = self.bucket_of[i]
            if stream is not None:
                st["streams"][b][stream.cuda_stream] = stream
            st["pending"][b] -= 1
            if st["pending"][b] == 0 and self.overlap and self.collective:
                if self.defer and self.params[0].is_cuda:
                    st["ready"].append((b, self._ready_events(b)))
                else:
                    self._launch(b)

    # ------------------------------------------------------------------ collectives
    def _bucket(self, b):
        o, n, _ = self.plan[b]
        return self.flat[o:o + n]

    def _ready_events(self, b):
        """Events on every stream that produced bucket b's gradients, recorded now (when its
        last gradient has just been enqueued)."""
        evs = []
        for s in self._step["streams"][b].values():
            ev = torch.cuda.Event()
            ev.record(s)
            evs.append((ev, s))
        return evs

    def _launch_ready(self):
        """Fork the all-reduces of the buckets completed at an earlier report.  Deferred by one
        report so that, in the captured graph, the next weight-gradient launch is captured
        first: it becomes the first child of the bucket's last producer and keeps that node's
        hardware queue, and the RCCL fork is a later child (the graph executor puts a node's
        first child on its parent's queue and later children on the next queues).
        Forked at once, the RCCL node was the first child and moved the weight-gradient chain
        onto the critical chain's queue: no overlap left (profiles/r05_final/dp_timeline.txt)."""
        st = self._step
        if not st or not st["ready"]:
            return
        ready, st["ready"] = st["ready"], []
        for b, evs in ready:
            self._launch(b, evs)

    def _comm_stream(self, capturing):
        st = self._comms.get(capturing)
        if st is None:
            st = self._comms[capturing] = torch.cuda.Stream(device=self.params[0].device)
        return st

    def _on_comm(self, waits, body, events=None):
        """Run `body` (which issues collectives in their synchronous form) on a communication
        stream that first waits on the streams `waits` (their current position) and on the
        (event, stream) pairs `events`: the capture-only stream while the current stream is
        capturing, else the eager one.  Returns the stream; the caller joins it (the caller's
        stream must wait on it before the gradients are read)."""
        capturing = torch.cuda.is_current_stream_capturing()
        comm = self._comm_stream(capturing)
        for s in waits:
            comm.wait_stream(s)
            ops.note_fork(comm, s, "RCCL stream")
        for ev, s in events or ():
            comm.wait_event(ev)
            ops.note_fork(comm, s, "RCCL stream")
        with torch.cuda.stream(comm):
            body()
        return comm

    def _launch(self, b, events=None):
        """One AVG (or, unaveraged, SUM) all-reduce of the bucket on the communication stream forked from the bucket's producers; the CALLER's stream
        joins it at the end of the backward (under hipGraph capture a forked stream must join
        the capture's origin stream directly: a wait on it from another forked stream crashes
        graph instantiation on this ROCm — tools/dp_capture_diag.py "kernel" vs "mainwait")."""
        bucket = self._bucket(b)
        if not self.params[0].is_cuda:  # CPU tensors (gloo tests)
            if self.average:
                bucket.mul_(1.0 / self.world)
            self._step["works"].append(dist.all_reduce(bucket, async_op=True))
            return

        avg = self.average and self.backend == "nccl"  # gloo has no AVG: pre-scale, then SUM

        def body():  # synchronous form: enqueued on the communication stream
            if self.average and not avg:
                bucket.mul_(1.0 / self.world)
            dist.all_reduce(bucket, op=dist.ReduceOp.AVG if avg else dist.ReduceOp.SUM)

        if events is None:
            comm = self._on_comm(self._step["streams"][b].values(), body)
        else:
            comm = self._on_comm((), body, events)
        self._step["comms"][comm.cuda_stream] = comm

    def _finish(self):
        # this callback runs before the side streams' join callbacks: the deferred LayerNorm
        # affine reductions report their parameters now
        ops.flush_held()
        ops.flush_deferred_affine()
        self._launch_ready()  # the last bucket(s)
        st, self._step = self._step, None
        if st is None:
            return
        # this callback may run before the weight-gradient side streams' own join callbacks:
        # order the caller's stream after every stream that produced a gradient
        cur = self._stream()
        if cur is not None:
            for s in st["producers"].values():
                if s.cuda_stream != cur.cuda_stream:
                    cur.wait_stream(s)
                    ops.note_join(cur, s)
        if self.plan is None:
            self._build_plan()
            self._fallback(list(range(len(self.params))))
            return
        if not st["fast"]:  # .grad already held gradients (accumulation): reduce them as they are
            self._fallback(list(range(len(self.params))))
            return
        missing = [b for b, n in enumerate(st["pending"]) if n != 0]
        if missing:
            raise RuntimeError(f"GradBuckets: buckets {missing} did not receive all their gradients this step "
                               "(the parameter set producing gradients changed after the first step)")
        for i, (o, n) in self.slot.items():  # .grad is the slot (whether or not autograd stole the view)
            p = self.params[i]
            if p.grad is None or p.grad.data_ptr() != self.flat[o:].data_ptr():
                p.grad = self.flat[o:o + n].view(p.shape)
        for work in st["works"]:
            work.wait()  # CPU (gloo) works: completes them
        for comm in st["comms"].values():  # GPU: the caller's stream joins the RCCL stream
            cur.wait_stream(comm)
            ops.note_join(cur, comm)
        self._fallback([i for i, p in enumerate(self.params) if i not in self.slot and p.grad is not None])

    def _build_plan(self):
        planned = [i for i in self._order if self._count[i] == 1]
        off, cur, buckets = 0, [], []
        start = 0
        for i in planned:
            n = self.params[i].numel()
            if cur and (off + n - start) * 4 > self.bucket_bytes:
                buckets.append((start, off - start, cur))
                start, cur = off, []
            self.slot[i] = (off, n)
            cur.append(i)
            off += -(-n // _ALIGN) * _ALIGN
        if cur:
            buckets.append((start, off - start, cur))
        self.plan = buckets
        for b, (_, _, idx) in enumerate(buckets):
            for i in idx:
                self.bucket_of[i] = b
        self.flat = torch.zeros(max(off, 1), device=self.params[0].device, dtype=torch.float32)

    def _fallback(self, idx):
        """All-reduce (and average) the gradients of parameters `idx` that hold one, in one
        flattened collective, on the current stream."""
        self.last_fallback = [i for i in idx if self.params[i].grad is not None]
        if not self.collective or not self.last_fallback:
            return
        grads = [self.params[i].grad for i in self.last_fallback]

        def body():
            flat = torch.cat([g.reshape(-1) for g in grads])
            dist.all_reduce(flat)
            if self.average:
                flat.mul_(1.0 / self.world)
            o = 0
            for g in grads:
                g.copy_(flat[o:o + g.numel()].view_as(g))
                o += g.numel()

        self._collective_here(body)

    def _collective_here(self, body):
        """`body` ordered on the current stream: on a communication stream (GPU) joined back
        into the current stream right away; directly (CPU tensors)."""
        if not self.params[0].is_cuda:
            body()
            return
        cur = torch.cuda.current_stream()
        comm = self._on_comm([cur], body)
        cur.wait_stream(comm)
        ops.note_join(cur, comm)

    # ------------------------------------------------------------------ non-overlapped mode
    def sync(self):
        """Without overlap: all-reduce the planned gradients (the flat buffer, in place) after
        the backward / graph replay.  A no-op in the overlapped mode or at world size 1."""
        if not self.collective:
            return
        if self.plan is None:  # no backward went through the ops sites: reduce .grad as it is
            self._fallback(list(range(len(self.params))))
            return
        if self.overlap:
            return

        def body():
            dist.all_reduce(self.flat)
            if self.average:
                self.flat.mul_(1.0 / self.world)

        self._collective_here(body)

    def quiesce(self):
        """Call before capturing a step into a hipGraph: completes every eager kernel and
        collective of the warm-up.  Capture runs in `thread_local` mode (ProcessGroupNCCL's
        watchdog thread queries events from ITS thread while the main thread captures), and
        nothing of the warm-up's autograd graphs may be alive (the caller drops its outputs: a
        captured backward that reused a warm-up AccumulateGrad node would fork into the
        warm-up's stream).  The watchdog may still list warm-up works when capture begins —
        harmless, because their events sit on the eager communication stream, which is never
        captured (see the module docstring)."""
        torch.cuda.synchronize()

    def bucket_sizes(self):
        return [n * 4 for _, n, _ in (self.plan or [])]


class GradAllReduce(GradBuckets):
    """Back-compatible name: the bucketed reducer, called after each step (`reducer()`)."""

    def __call__(self):
        self.sync()


def gathered_mean(local):
    """Mean over ranks of every rank's `local` tensor, summed in rank order after an eager
    all_gather (outside any capture): the reference value for the averaged buckets of a
    data-parallel step (bench.py prints max |buckets - this| at world size > 1).  Over gloo
    the gather runs on host copies."""
    world = dist.get_world_size()
    on_host = dist.get_backend() != "nccl"
    src = local.detach().cpu() if on_host else local.detach().contiguous()
    parts = [torch.empty_like(src) for _ in range(world)]
    dist.all_gather(parts, src)
    acc = parts[0].clone()
    for t in parts[1:]:
        acc.add_(t)
    return acc.div_(world).to(local.device)
