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
