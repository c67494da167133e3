"""One training step of the reference's train.py hot loop (train.py:97-135, 250-327 REFINE;
140-249 ALL), on librod kernels:

  normalise -> corner->centre -> anchor matching (per image, batched on the GPU) ->
  network forward -> refine loss (+ det/clf loss in ALL) -> backward -> [DP all-reduce]
  -> SGD with clip-by-value.

Data-parallel: one process per GPU, the per-image batch sharded across ranks; the
flat gradient buffer is all-reduced (sum) over RCCL and losses are normalised by the
GLOBAL batch so the sum equals the single-process gradient (the reference divides by
bs, net_tools.py:513).  Clipping happens after the reduction (net_tools.py:649).
BatchNorm statistics are per rank by default (documented deviation) or, with
sync_bn=True, merged over the global batch (rod.ddp.SyncBatchNorm); the hard negatives are
selected over the global batch (counts + radix histograms all-reduced, ops.hnm_lockstep).
"""
from __future__ import annotations

import numpy as np
import torch

import config
from nets.catch_net import CatchNet, factory
from rod import graph, ops
from utils import net_tools
from utils.common_tools import cornerBboxes_2_centerBboxes


class Trainer:
    MAX_GRAPHS = 4   # captured step graphs kept (one per batch signature), oldest dropped first

    def __init__(self, img_size, batch_size, dtype=torch.bfloat16, train_range=config.train_range.REFINE,
                 learning_rate=1e-3, device='cuda', fix_refine=True, seed=0, world_size=1, reducer=None,
                 deconv_method=config.deconv_method.LEARN_HALF, merge_method=config.merge_method.ADD,
                 sync_bn=False, backbone_name='mobilenet_v2',
                 process_backbone_method=config.process_backbone_method.NONE):
        self.img_size = tuple(img_size)
        self.batch_size = batch_size          # per-rank batch
        self.world_size = world_size
        self.dtype = dtype
        self.device = torch.device(device)
        config.img_size = self.img_size       # init_anchor reads config.img_size (net_tools.py:37-38)
        self.config_dict = {'train_range': train_range,
                            'process_backbone_method': process_backbone_method,
                            'deconv_method': deconv_method,     # train.py:131-133 defaults
                            'merge_method': merge_method}
        self.backbone_name = backbone_name
        self.net = CatchNet(backbone_name, self.config_dict, self.device, seed)
        layer_n = len(config.extract_feat_name[backbone_name])
        self.anchors = net_tools.anchors_all_layer(self.img_size, config.feat_sizes(self.img_size, backbone_name),
                                                   net_tools.init_anchor(layer_n))
        self.table = net_tools.anchor_table(self.anchors, self.device)
        store = self.net.store
        if train_range is config.train_range.ALL and fix_refine:
            import re
            pat = re.compile(r'^((?!(backbone|refine)).)*$')   # train.py:160-163
            store.set_trainable(lambda n: bool(pat.match(n)))
        self.opt = net_tools.optimizer(store, batch_size * world_size, learning_rate)
        self.reducer = reducer
        if reducer is not None and hasattr(reducer, 'attach'):
            reducer.attach(store)  # buckets over the trainable parameters (rod.ddp)
        # hard negatives over the global batch (net_tools.py:557-587)
        # (a reducer is only handed in by a data-parallel job; a 1-rank group exercises the same
        # exchange path, e.g. the graph-capture test)
        dp = reducer is not None
        net_tools.HNM_EXCHANGE = (reducer.hnm_allreduce, world_size) \
            if dp and hasattr(reducer, 'hnm_allreduce') else None
        self.train_range = train_range
        self.fix_refine = fix_refine
        # BatchNorm over the global batch (opt-in; per-rank statistics otherwise)
        self.sync_bn = bool(sync_bn and (world_size > 1 or dp))
        if self.sync_bn:
            from rod.ddp import SyncBatchNorm
            ops.SYNC_BN = SyncBatchNorm(world_size, getattr(reducer, 'group', None),
                                        comm=getattr(reducer, 'comm', None))
        else:
            ops.SYNC_BN = None
        # weight gradients beside the backward-data chain (opt-in, ROD_ENABLE=side; single
        # process only: under DP the gradient buckets are reduced from inside backward).
        # Measured slower: 24.42 -> 24.93 ms per graphed step
        self._side = world_size == 1 and reducer is None and "side" in ops._ENABLE
        rank = torch.distributed.get_rank() if world_size > 1 and torch.distributed.is_initialized() else 0
        ops.DROPOUT_RANK[:] = [rank, world_size]
        self._eager_steps = 0
        self._dropout_seen = False   # the step draws dropout masks (vgg_16 training): never graphed

    def step(self, img_u8, gt_corner, gt_labels, gt_n):
        losses = self._compute(img_u8, gt_corner, gt_labels, gt_n)
        if self.reducer is not None:
            self.reducer(self.net.store.flat_grad)
        self.opt.step()
        self._eager_steps += 1
        return losses

    def _compute(self, img_u8, gt_corner, gt_labels, gt_n):
        """Forward + backward of one step: the parameter gradients in the flat buffer (the
        data-parallel buckets launch from inside backward unless the reducer is deferred)."""
        calls = ops._DROPOUT_CALLS[0]
        losses = self.losses(img_u8, gt_corner, gt_labels, gt_n)
        self._dropout_seen |= ops._DROPOUT_CALLS[0] != calls
        if self._side:
            ops.SIDE.backward(losses[0], self.device)
        else:
            # the weight-gradient slab sums are batched into a few launches at the end
            ops.SLAB.begin()
            try:
                graph.backward(losses[0])
            finally:
                ops.SLAB.end()
        return losses

    def graph_mode(self):
        """How step_graphed runs this trainer's step:
        'full'  — the whole step is one graph: single process, or data parallel through the
                  library's RCCL communicator (rod.ddp native reducer, the N > 1 default over
                  RCCL): the bucketed all-reduces on their side stream (overlapping backward),
                  the hard-negative exchange and the SyncBatchNorm gathers are captured with
                  the kernels;
        'split' — data parallel over torch.distributed (gloo: the CPU rehearsal): forward +
                  backward (no collective inside: REFINE mode without SyncBatchNorm) replay as
                  a graph, then the gradient all-reduce and SGD are issued eagerly;
        'eager' — torch.distributed steps with collectives inside forward/backward (ALL mode's
                  global hard negatives, SyncBatchNorm); dropout."""
        if self._dropout_seen:
            return 'eager'
        if self.reducer is None or getattr(self.reducer, 'native', False):
            return 'full'
        hnm = self.train_range is not config.train_range.REFINE and net_tools.HNM_EXCHANGE is not None
        mid = self.sync_bn or hnm
        return 'eager' if mid or not hasattr(self.reducer, 'defer') else 'split'

    def step_graphed(self, img_u8, gt_corner, gt_labels, gt_n):
        """One training step replayed as a HIP graph: the whole forward / backward / SGD launch
        sequence (~960 kernels) is captured once on the first call after an eager step (which did
        the lazy set-up: anchor tables, weight-layout cache, workspaces) and replayed from static
        input buffers, so no per-kernel host dispatch remains.  Every call runs exactly one step;
        the results are bit-identical to step() (same kernels, same order).  Host-side step state
        (opt.global_step) advances once per replay.  A step that draws dropout masks (the vgg_16
        backbone in training) runs eager: its mask seed is a host counter that a replay would
        freeze.

        Data parallel through the library's communicator: the bucketed gradient all-reduces that
        backward launches (on the communication stream, forked from and joined back into the
        compute stream by events), the hard-negative exchange and the SyncBatchNorm all-gathers
        are captured with the kernels and replay with them.  No collective of torch.distributed
        runs in the step, so RCCL's host watchdog has nothing to poll while the step is captured.
        gloo runs on the host and cannot be captured: with it only forward + backward replay.

        Graphs: one per batch signature (the TFRecord source pads the boxes to a fixed count, so
        a run normally has one), each on its own memory pool — a graph's outputs (`out`) stay
        valid until that same graph replays again, whatever other signature replays between.
        Captures run in thread_local mode: a prefetching data source may allocate and copy on
        its own thread meanwhile (rod.dataio), which is legal outside the capturing thread."""
        mode = self.graph_mode()
        if self._eager_steps == 0 or mode == 'eager':
            return self.step(img_u8, gt_corner, gt_labels, gt_n)
        new = (img_u8, gt_corner, gt_labels, gt_n)
        key = tuple((tuple(t.shape), t.dtype) for t in new)
        graphs = self.__dict__.setdefault('_graphs', {})
        if key not in graphs:
            if len(graphs) >= self.MAX_GRAPHS:
                graphs.pop(next(iter(graphs)))   # its graph and pool are freed with it
            static = tuple(t.clone() for t in new)
            self.net.store.build_prep_tables()   # host -> device set-up stays outside the capture
            g = torch.cuda.CUDAGraph()
            torch.cuda.synchronize()
            st = self.net.store
            gstep, eager, version = self.opt.global_step, self._eager_steps, st.version
            if mode == 'split':
                self.reducer.defer = True   # no bucket launches from inside the captured backward
            try:
                with torch.cuda.graph(g, pool=torch.cuda.graph_pool_handle(), capture_error_mode='thread_local'):
                    out = self.step(*static) if mode == 'full' else self._compute(*static)
            finally:
                if mode == 'split':
                    self.reducer.defer = False
            # the capture recorded the step without running it: host counters as before
            self.opt.global_step, self._eager_steps, st.version = gstep, eager, version
            graphs[key] = (g, static, out)
        g, static, out = graphs[key]
        self._graph = graphs[key]
        for a, b in zip(static, new):
            if a.data_ptr() != b.data_ptr():
                a.copy_(b)
        g.replay()
        if mode == 'split':
            self.reducer(self.net.store.flat_grad)   # every bucket, back to back, then SGD
            self.opt.step()
            return out
        self.opt.global_step += 1
        self.net.store.version += 1   # the replay's SGD changed the parameters (derived layouts stale)
        return out

    def losses(self, img_u8, gt_corner, gt_labels, gt_n):
        """Forward of one step: (training loss, [refine, det, clf] in ALL mode)."""
        if img_u8.is_floating_point():   # already (2/255)x - 1 (fused into rod_augment_images)
            x = ops.cast(img_u8, self.dtype)
        else:
            x = ops.normalize_image(img_u8, self.dtype)             # (2/255)x - 1
        center = cornerBboxes_2_centerBboxes(gt_corner)              # train.py:109
        tg = net_tools.refine_groundtruth(self.anchors, center, gt_labels, config.refine_method.JACCARD_BIGGER,
                                          n_boxes=gt_n)
        out = factory(x, self.backbone_name, True, self.config_dict, self.dtype, net=self.net).get_output()
        scale = float(self.batch_size * self.world_size)
        if self.train_range is config.train_range.REFINE:
            loss = net_tools.refine_loss(out, tg[0], tg[3], targets=tg, scale=scale)
            losses = (loss,)
        else:
            refine_out, det_out, clf_out = out
            self.last_out = out
            rflat = [None, None]
            if not self.fix_refine:
                # refine_out feeds the refine loss AND the ODM targets / IoU factor (train.py:144-151,
                # total_loss = refine + det + clf): one concatenation, two aliases whose gradients
                # meet in rod_add
                rflat = list(graph.fork(ops.levels_concat(refine_out, 4), 2))
            r_loss = net_tools.refine_loss(refine_out, tg[0], tg[3], targets=tg, scale=scale, refine_flat=rflat[0])
            dgt = net_tools.det_groundtruth(refine_out, tg[0], tg[1], tg[2], tg[3], self.anchors, targets=tg,
                                            refine_flat=rflat[1])
            d_loss, c_loss = net_tools.det_clf_loss(refine_out, clf_out, det_out, dgt, dgt[1], dgt[2], dgt[3],
                                                    scale=scale)
            loss = graph.scalar_sum(d_loss, c_loss) if self.fix_refine else graph.scalar_sum(r_loss, d_loss, c_loss)
            losses = (loss, r_loss, d_loss, c_loss)
            self.last_targets = (tg, dgt)
        return losses
