"""Whole-step HIP graph capture.

A training step of this model is ~1500 small kernel launches; issued one by one from
Python the host, not the GPU, sets the step time.  `StepGraph` records the step once as
a short sequence of hipGraphs (one memory pool) and replays it with one launch per
segment.  Host work that must stay outside a graph -- RCCL all-reduces of the flat
gradient buffers and of the sync_codebook statistics, learning-rate schedulers --
runs eagerly between / before the segments.

Everything inside a segment must be capturable: no host synchronisation, device-side
randomness only (the dropout seed advances on the device, layer-dropout decisions are
drawn on the device under `rng.device_decisions()`), fixed input buffers.
"""
import gc

import torch

from . import rng, streams
from ._native import call


class StepGraph:
    """segments[i]() are captured in order; between[i]() (eager, may be None) runs after
    segment i on every replay.  `warmup` eager steps run on a side stream first (lazy
    initialisation must not happen inside a capture); they are real steps."""

    def __init__(self, segments, between=None, warmup=2, before=None):
        self.segments = list(segments)
        self.between = list(between or [None] * len(self.segments))
        self.before = before
        self.warmup = warmup
        self.graphs = None
        self.outputs = None

    def _eager(self):
        if self.before is not None:
            self.before()
        outs = []
        for seg, btw in zip(self.segments, self.between):
            outs.append(seg())
            streams.join(backward_done=True)
            if btw is not None:
                btw()
        return outs

    def capture(self):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side), rng.device_decisions():
            for _ in range(self.warmup):
                self._eager()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        pool = torch.cuda.graph_pool_handle()
        self.graphs, self.outputs = [], []
        call("tvq_counter_capture", 1)  # finish-counter slots of the graph stay reserved
        # no garbage collection inside a capture: collecting an unreachable graph of an
        # earlier capture (reference cycles) destroys it, which HIP refuses while a stream
        # is capturing
        gc_on = gc.isenabled()
        gc.collect()
        gc.disable()
        try:
            with rng.device_decisions():
                for seg in self.segments:
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, pool=pool):
                        out = seg()
                        streams.join(backward_done=True)  # side-stream branches rejoin
                    self.graphs.append(g)
                    self.outputs.append(out)
        finally:
            call("tvq_counter_capture", 0)
            if gc_on:
                gc.enable()
        return self

    def replay(self):
        if self.before is not None:
            self.before()
        for g, btw in zip(self.graphs, self.between):
            g.replay()
            if btw is not None:
                btw()
        return self.outputs


class BranchStepGraph:
    """A step whose independent parts run as separate graphs on their own streams, each
    followed by its own eager exchange, then a final graph:

        before(); pre()                                  eager, current stream
        branch i: graph_i ; after_i()                    stream S_i (waits for pre)
        final graph                                      current stream (waits for every S_i)

    The DP trainer's form (bench.JointTrainer at world > 1): stage1's and stage2's
    forward+backward are the branches, each branch's all-reduces start as soon as its own
    backward ends -- while the other branch still computes -- and the optimizers are the
    final graph.  Each graph has its own memory pool: branch graphs replay concurrently, so
    their allocations must not alias (graphs sharing a pool must replay in capture order).

    replay_order: the order the branches (and their exchanges) are enqueued at replay.  The
    collectives of one process group run in host-issue order on its communication stream
    (torch's ProcessGroupNCCL stream; the same order on every rank, so RCCL cannot
    deadlock), so the branch that finishes first must be issued first for its exchange to
    overlap the other branch's compute.  Capture always runs in list order.
    """

    def __init__(self, pre, branches, afters, final, warmup=2, before=None, replay_order=None):
        self.pre, self.branches, self.afters = pre, list(branches), list(afters)
        self.final, self.before, self.warmup = final, before, warmup
        self.order = list(replay_order) if replay_order is not None else list(range(len(self.branches)))
        assert sorted(self.order) == list(range(len(self.branches))), "replay_order: a permutation"
        self.graphs = self.final_graph = None
        self.outputs = None
        self._streams = None

    def _eager(self):
        if self.before is not None:
            self.before()
        self.pre()
        outs = []
        for br, aft in zip(self.branches, self.afters):
            outs.append(br())
            streams.join(backward_done=True)
            if aft is not None:
                aft()
        self.final()
        streams.join(backward_done=True)
        return outs

    def capture(self):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side), rng.device_decisions():
            for _ in range(self.warmup):
                self._eager()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graphs, self.outputs = [], []
        call("tvq_counter_capture", 1)
        gc_on = gc.isenabled()
        gc.collect()
        gc.disable()
        try:
            with rng.device_decisions():
                # pre() is not captured (it runs eagerly before every replay); the branches
                # restore any host state it sets (bench: rng.restart_calls())
                for br in self.branches:
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, pool=torch.cuda.graph_pool_handle()):
                        out = br()
                        streams.join(backward_done=True)
                    self.graphs.append(g)
                    self.outputs.append(out)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=torch.cuda.graph_pool_handle()):
                    self.final()
                    streams.join(backward_done=True)
                self.final_graph = g
        finally:
            call("tvq_counter_capture", 0)
            if gc_on:
                gc.enable()
        torch.cuda.synchronize()
        self._streams = [torch.cuda.Stream() for _ in self.branches]
        return self

    def replay(self):
        if self.before is not None:
            self.before()
        cur = torch.cuda.current_stream()
        self.pre()
        for i in self.order:
            g, aft, st = self.graphs[i], self.afters[i], self._streams[i]
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                g.replay()
                if aft is not None:
                    aft()
        for st in self._streams:
            cur.wait_stream(st)
        self.final_graph.replay()
        return self.outputs
