"""One training step with the semantics of train_multi_gpu.py:train_one_step (:56-129).

The step is: forward -> (discriminator on real / fake) -> total_loss -> Balancer -> ONE backward
over [output, loss_w] with grads [balanced, 1] -> RCCL all-reduce of the flat generator grads
(world > 1) -> Adam; then, for the GAN configs, the discriminator update. It never reads a
device value on the host, so consecutive steps queue back to back.

The discriminator runs forward ONCE per step on the real and on the fake audio. The reference
runs it twice on each (train_multi_gpu.py:62-63 in the generator phase, :114-116 in the
discriminator phase); the discriminator's weights and the generator output are unchanged in
between (only the generator's Adam step runs there), so the second pair of forwards is
value-identical recomputation. Here the generator phase differentiates the shared graph w.r.t.
the audio only and the discriminator phase w.r.t. the weights only (ops.DiscGradMode); the
fake branch is fed a detached leaf of the output, so the discriminator phase never reaches the
generator graph, as the reference's output.detach() (:116).

Documented deviations: #7 a single combined backward (identical at
world_size 1; at world_size > 1 the commit-loss grads are all-reduced too, true DP);
#9 the discriminator is trained with an explicit probability instead of eval(bool).
"""
import contextlib
import os
import random

import torch

from .balancer import Balancer
from . import distrib
from .losses import total_loss, disc_loss
from .model import EncodecModel
from .ops import DiscGradMode, WnBatch, defer_codebook_sync
from .optim import FlatAdam
from .scheduler import WarmupCosineLrScheduler

def _noop():
    pass


DEFAULT_WEIGHTS = {'l_t': 0.1, 'l_f': 1, 'l_g': 3, 'l_feat': 3}  # config/config.yaml:55-60


class Trainer:
    def __init__(self, model: EncodecModel, disc=None, lr=3e-4, disc_lr=3e-4, betas=(0.5, 0.9),
                 weights=None, max_iter=100000, warmup_iter=0, disc_prob=1.0, sample_rate=24000,
                 scheduler=True, balancer_kwargs=None, graphs=False, ddp_commit_local=False,
                 segmented=None):
        self.model = model
        # segmented: the device part as the data-parallel list of segments (split backward,
        # one HIP graph per segment) even at world 1, where the collectives between them are
        # no-ops. None = segmented exactly when distributed.
        self.segmented = segmented
        self._seg_hook = None  # diagnostics: called with the segment index after each segment
        # ddp_commit_local: the reference's exact DDP semantics (train_multi_gpu.py:86-95, SURVEY
        # quirk 7): the commit loss's grads are added AFTER the all-reduce, so they stay rank-local
        # and the ranks' weights drift apart. Off (default): one backward, true data parallelism.
        self.ddp_commit_local = ddp_commit_local
        self.disc = disc
        self.sample_rate = sample_rate
        if distrib.is_distributed():
            distrib.broadcast_tensors(model.parameters())
            if disc is not None:
                distrib.broadcast_tensors(disc.parameters())
        self.opt = FlatAdam(model.parameters(), lr=lr, betas=betas)
        self.opt_d = FlatAdam(disc.parameters(), lr=disc_lr, betas=betas) if disc is not None else None
        w = dict(weights or DEFAULT_WEIGHTS)
        if disc is None:
            w = {k: w[k] for k in ('l_t', 'l_f')}
        self.balancer = Balancer(w, **(balancer_kwargs or {}))
        self.sched = self.sched_d = None
        if scheduler:
            self.sched = WarmupCosineLrScheduler(self.opt, max_iter=max_iter, eta_ratio=0.1,
                                                 warmup_iter=warmup_iter, warmup_ratio=1e-4)
            if disc is not None:
                self.sched_d = WarmupCosineLrScheduler(self.opt_d, max_iter=max_iter, eta_ratio=0.1,
                                                       warmup_iter=warmup_iter, warmup_ratio=1e-4)
        self.disc_prob = disc_prob
        # the step feeds the feature maps to the losses only (FeatFn), so the Conv2d backward may
        # pass pre-activation grads between layers (DiscGradMode.premask) wherever the bwd-data
        # epilogue reads the input map anyway (the feature-matching term); ENCX_PREMASK=0 off
        self.disc_mode = DiscGradMode(premask=os.environ.get('ENCX_PREMASK', '1') != '0')
        # every weight norm of a step as one launch per model forward and per backward
        # (ops.WnBatch); ENCX_WN_BATCH=0 keeps the per-layer launches
        self.wn = WnBatch() if os.environ.get('ENCX_WN_BATCH', '1') != '0' else None
        self.graphs = graphs
        self._graphs = {}
        self._pool = None  # one HIP-graph memory pool shared by every captured key
        self.max_graph_keys = 8  # keys past this many run eagerly (their pool memory is bounded)
        dec = [p for p in model.decoder.parameters() if p.requires_grad]
        self._dec_span = self.opt.span(dec) if dec else None
        self._sync = None  # the persistent LSTM's error watch (_watch_sync)

    # ------------------------------------------------------------------ step
    # step() = host part (draw the bandwidth and the discriminator coin, advance the optimiser step
    # counts and write their scalars) + device part. The device part is a list of segments with
    # the cross-rank collectives between them (world > 1; at world 1 every collective is None):
    #   gen     zero grads, generator forward (synced codebooks: the per-code sums, deferred)
    #     -- start the all-reduce of the codebook sums (async)
    #   losses  discriminator on real / fake, losses, per-loss grads, balancer statistics
    #     -- all-reduce the balancer statistics (nl + 1 floats)
    #   dec     balancer scales + combine; backward output -> decoder weights and the decoder
    #           input's grad (the whole backward when the model is segmented or world is 1)
    #     -- start the all-reduce of the decoder's grad bucket (async)
    #   enc     backward (quantized, loss_w) -> encoder
    #     -- start the all-reduce of the encoder's grad bucket (async)
    #   disc    discriminator loss + its weight-grad backward (independent of the generator
    #           update, so the generator's buckets reduce underneath it)
    #     -- start the discriminator's all-reduce; wait for every collective of the step
    #   opt     codebook EMA from the reduced sums, generator Adam, discriminator Adam
    # The reference's order is generator Adam, then the discriminator phase (train_multi_gpu.py
    # :95, :112-124); the discriminator phase reads neither the generator's weights nor its
    # grads, so running its backward first changes no value.
    # With graphs=True each (bandwidth, coin, shape) key runs eagerly once, is then captured into
    # HIP graphs (one per segment between collectives; world 1: the whole step is one graph), and
    # is replayed after. All keys share one memory pool: replays never overlap, and every tensor
    # a replay reads is written earlier in the same replay (inputs are copied into a buffer
    # outside the pool; losses are copied out of it on return).
    def step(self, x):
        model, disc = self.model, self.disc
        model.train()
        if disc is not None:
            disc.train()
        bw = model._pick_bandwidth(x.device)
        train_d = disc is not None and self._pick_train_d(x.device)
        self.opt.prepare()
        if train_d:
            self.opt_d.prepare()
        key = (bw, train_d, tuple(x.shape))
        # At world > 1 the step would be cut into segments around the collectives, one graph
        # each. That is opt-in (ENCX_DP_GRAPHS=1): round 3 recorded replays drifting from the
        # eager step at world 2 (profiles/r03/dp_graph_replay_diag.txt) with no cause proven,
        # and no multi-GPU RCCL run has compared replays with eager steps.
        if self.graphs and (not distrib.is_distributed() or os.environ.get('ENCX_DP_GRAPHS', '0') == '1') \
                and self._graph_ok(key):
            out = self._graph_step(key, x)
        else:
            out = self._run(x, bw, train_d)
        self._watch_sync(x.device)
        if os.environ.get('ENCX_CHECK_SYNC', '0') == '1':
            self.check_sync()  # debugging: wait for this step and check it now
        if self.sched is not None:
            self.sched.step()
        if self.sched_d is not None:
            self.sched_d.step()
        return out

    # The persistent LSTM kernels hand frames between workgroups through counters with bounded
    # spins; a spin that times out (workgroups not co-resident, e.g. a foreign kernel holding CUs)
    # leaves that launch's results garbage and bumps a per-device error word (csrc/lstm.hip). After
    # every step one tiny kernel folds the word into a device counter, which is copied to pinned
    # memory asynchronously; the next step() reads the copy if it has landed (no sync, no stall of
    # the queue) and raises on a nonzero count. check_sync() waits for the last step's copy.
    def _watch_sync(self, device):
        from ._lib import call, ptr, stream
        w = self._sync
        if w is None:
            w = self._sync = [torch.zeros(1, dtype=torch.int32, device=device),
                              torch.zeros(1, dtype=torch.int32).pin_memory(), torch.cuda.Event(), False]
        dev, host, ev, pending = w
        if pending and ev.query():
            self._raise_sync(int(host[0]))
        call('encx_lstm_sync_read', ptr(dev), stream())
        host.copy_(dev, non_blocking=True)
        ev.record()
        w[3] = True

    def check_sync(self):
        """Wait for the last step's error-word copy and raise if any LSTM hand-off failed."""
        w = self._sync
        if w is not None and w[3]:
            w[2].synchronize()
            self._raise_sync(int(w[1][0]))

    @staticmethod
    def _raise_sync(n):
        if n:
            raise RuntimeError(f'encx: {n} persistent-LSTM hand-off failures (spin timeouts or counters off '
                               'their count) since training started: those steps\' LSTM results are garbage '
                               '(workgroups not co-resident? another persistent launch on the GPU?)')

    def _pick_train_d(self, device):
        """train_multi_gpu.py:105-110. disc_prob None = the reference's short-circuit (the flag
        off, or a warmup epoch): no random draw, so Python's RNG stream stays the reference's."""
        if self.disc_prob is None:
            return False
        train_d = random.random() < self.disc_prob
        if distrib.is_distributed() and self.disc_prob < 1.0:
            t = torch.tensor([train_d], device=device)
            torch.distributed.broadcast(t, 0)
            train_d = bool(t.item())
        return train_d

    def _segments(self, x, bw, train_d):
        """The device part as (segment, collective) pairs; state flows through `c`."""
        c = {}
        dist = distrib.is_distributed()
        seg = dist if self.segmented is None else bool(self.segmented)
        split = seg and self._dec_span is not None and self.model.segment is None
        local = dist and self.ddp_commit_local
        if local and not split:
            raise ValueError('encx Trainer: ddp_commit_local needs an unsegmented model')
        works = []

        wn = self.wn
        fwd = (lambda grp: wn.forward(grp)) if wn is not None else (lambda grp: contextlib.nullcontext())
        bwd = (lambda: wn.backward()) if wn is not None else contextlib.nullcontext

        # synced codebooks: the EMA sums' all-reduce is deferred to a collective between segments
        # only for a one-frame model; with segments (48 kHz) frame f + 1 must quantise with the
        # codebooks synced after frame f, so the RVQ forward all-reduces in place (eager step)
        defer = (lambda: defer_codebook_sync(c['cb'])) if self.model.segment is None else contextlib.nullcontext

        def seg_gen():
            self.opt.zero_grad()
            c['cb'] = []
            with fwd('gen'), defer():
                y, loss_w, _ = self.model(x, bandwidth=bw, split=split)
            c['y'], c['loss_w'] = y, loss_w
            c['y_out'] = self.last_y = y.detach()  # the step's generator output (tests' L1 sign audit)
            c['split'] = self.model.last_split

        def coll_gen():
            works.extend(torch.distributed.all_reduce(e.sums, async_op=True) for e in c['cb'])

        def seg_losses():
            y = c['y']
            if self.disc is not None:
                # generator phase: the balancer's autograd.grad calls differentiate the shared
                # discriminator graph w.r.t. the fake audio only
                self.disc_mode.set(params=False, input=True)
                self.disc_mode.reuse_weights(True)  # same weights for both forwards
                yd = y.detach().requires_grad_()
                with fwd('disc'):
                    c['logits_real'], fmap_real = self.disc(x, mode=self.disc_mode)
                    c['logits_fake'], fmap_fake = self.disc(yd, mode=self.disc_mode)
                self.disc_mode.reuse_weights(False)
                losses = total_loss(fmap_real, c['logits_fake'], fmap_fake, x, yd, self.sample_rate)
                wrt = yd
            else:
                losses = total_loss(None, None, None, x, y, self.sample_rate)
                wrt = y
            c['losses'] = losses
            c['loss_grads'] = self.last_loss_grads = self.balancer.grads(losses, wrt)
            self.balancer.combine_start(c['loss_grads'])

        def seg_dec():
            out_grad = self.balancer.combine_finish()
            c['out_grad'] = self.last_out_grad = out_grad  # (tests' diagnostics)
            y, loss_w = c.pop('y'), c['loss_w']
            with bwd():
                if c['split'] is not None:
                    torch.autograd.backward([y], [out_grad])
                else:
                    torch.autograd.backward([y, loss_w], [out_grad, torch.ones_like(loss_w)])

        def coll_dec():
            works.append(self.opt.reduce_async(*self._dec_span))

        def seg_enc():
            q, leaf = c.pop('split')
            loss_w = c['loss_w']
            with bwd():
                if local:  # the balanced grads only; the commit backward follows the all-reduce
                    torch.autograd.backward([q], [leaf.grad], retain_graph=True)
                else:
                    torch.autograd.backward([q, loss_w], [leaf.grad, torch.ones_like(loss_w)])

        def coll_enc():
            # everything outside the decoder's bucket: [0, dec start) and, should any generator
            # parameter sit after the decoder in the flat buffer, [dec end, numel)
            n = self.opt.flat_grad.numel()
            a, b = self._dec_span if split else (n, n)
            if a > 0:
                works.append(self.opt.reduce_async(0, a))
            if b < n:
                works.append(self.opt.reduce_async(b, n))

        def seg_disc():
            # values only: the loss tensors would keep their graphs (the discriminator's
            # activations) alive for as long as the caller -- or a captured key -- holds them
            out = {k: v.detach() for k, v in c.pop('losses').items()}
            out['loss_w'] = c['loss_w'].detach()
            if train_d:
                # discriminator phase on the same graph: weight grads only (train_multi_gpu.py:112-124)
                self.disc_mode.set(params=True, input=False)
                self.opt_d.zero_grad()
                out['l_d'] = disc_loss(c.pop('logits_real'), c.pop('logits_fake'))
                with bwd():
                    out['l_d'].backward()
                out['l_d'] = out['l_d'].detach()
            c['out'] = out

        def coll_disc():
            if train_d:
                works.append(self.opt_d.reduce_async())
            for w in works:
                w.wait()
            works.clear()

        def seg_opt():
            for e in c['cb']:
                e.apply()  # the EMA codebook update from the rank-summed code sums
            if dist:
                self.opt.flat_grad.div_(distrib.world_size())
            if local:  # loss_w.backward() (train_multi_gpu.py:94): rank-local commit grads
                loss_w = c['loss_w']
                with bwd():
                    torch.autograd.backward([loss_w], [torch.ones_like(loss_w)])
            self.opt.launch()
            if train_d:
                if dist:
                    self.opt_d.flat_grad.div_(distrib.world_size())
                self.opt_d.launch()

        if not seg:
            segs = [seg_gen, seg_losses, seg_dec, seg_disc, seg_opt]
            return [(lambda: [s() for s in segs], None)], c
        if not dist:  # world 1, segmented on request: the same segments, no collectives
            return [(seg_gen, None), (seg_losses, None), (seg_dec, None),
                    (seg_enc if split else _noop, None), (seg_disc, None), (seg_opt, None)], c
        return [(seg_gen, coll_gen if self.model.quantizer.sync_codebooks else None),
                (seg_losses, self.balancer.reduce_stats),
                (seg_dec, coll_dec if split else None),
                (seg_enc if split else _noop, coll_enc),
                (seg_disc, coll_disc),
                (seg_opt, None)], c

    def _run(self, x, bw, train_d):
        segs, c = self._segments(x, bw, train_d)
        for i, (seg, coll) in enumerate(segs):
            seg()
            if coll is not None:
                coll()
            if self._seg_hook is not None:
                self._seg_hook(i, c)
        return c['out']

    def _graph_ok(self, key):
        from ._lib import lib
        if lib.encx_prof_enabled() or self.balancer.monitor:
            return False  # profiler events / the monitor's host read are not capturable
        if distrib.is_distributed() and self.model.quantizer.sync_codebooks and self.model.segment is not None:
            return False  # the codebook all-reduce runs inside the forward (seg_gen): not capturable
        return key in self._graphs or len(self._graphs) < self.max_graph_keys

    def _graph_step(self, key, x):
        ent = self._graphs.get(key)
        if ent is None:
            # first occurrence: eager (kmeans init, lazily built tables and the balancer state
            # happen here, outside any capture)
            self._graphs[key] = 'warm'
            return self._run(x, key[0], key[1])
        if ent == 'warm':  # second occurrence: capture, which also runs this step
            ent = self._graphs[key] = self._capture(key, x)
        else:
            graphs, colls, xs, out, codes, cap_c = ent
            xs.copy_(x)
            for i, (g, coll) in enumerate(zip(graphs, colls)):
                if g is not None:
                    g.replay()
                if coll is not None:
                    coll()
                if self._seg_hook is not None:
                    self._seg_hook(i, cap_c)
        out = ent[3]
        # this key's graphs rewrite its own codes tensor (held by the entry, so its pool block is
        # never handed to another key); after another key ran, last_codes must point back at it
        self.model.last_codes, self.model.seg_codes = ent[4]
        self.last_y = ent[5]['y_out']
        self.last_loss_grads, self.last_out_grad = ent[5]['loss_grads'], ent[5]['out_grad']
        # the replayed graphs rewrite `out` in place: hand the caller a copy of this step's values
        names = list(out)
        vals = torch.cat([out[k].detach().reshape(-1)[:1] for k in names])
        return {k: vals[i] for i, k in enumerate(names)}

    def _capture(self, key, x):
        xs = x.detach().clone()
        segs, c = self._segments(xs, key[0], key[1])
        torch.cuda.synchronize()
        if self._pool is None:
            self._pool = torch.cuda.graph_pool_handle()
        graphs, colls, pending = [], [], []
        for seg, coll in segs:
            g = None
            if seg is not _noop:  # an empty segment (no split backward) is not captured
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=self._pool):
                    seg()
                pending.append(g)
            graphs.append(g)
            colls.append(coll)
            if coll is not None:
                # capture only records: run every segment captured since the last collective for
                # real (in order: a segment without a collective of its own still feeds the next),
                # then the collective, which the next capture does not depend on
                for pg in pending:
                    pg.replay()
                pending.clear()
                coll()
        for pg in pending:
            pg.replay()
        if self._seg_hook is not None:
            self._seg_hook(len(segs) - 1, c)
        return graphs, colls, xs, c['out'], (self.model.last_codes, self.model.seg_codes), c

    # ------------------------------------------------------------------ checkpoints
    def state_dicts(self):
        """The four state dicts the reference checkpoints (utils.py:132-148)."""
        return {'optimizer': self.opt.state_dict(),
                'scheduler': self.sched.state_dict() if self.sched is not None else None,
                'disc_optimizer': self.opt_d.state_dict() if self.opt_d is not None else None,
                'disc_scheduler': self.sched_d.state_dict() if self.sched_d is not None else None}

    def load_state_dicts(self, optimizer=None, scheduler=None, disc_optimizer=None, disc_scheduler=None):
        """train_multi_gpu.py:303-307."""
        if optimizer is not None:
            self.opt.load_state_dict(optimizer)
        if scheduler is not None and self.sched is not None:
            self.sched.load_state_dict(scheduler)
        if disc_optimizer is not None and self.opt_d is not None:
            self.opt_d.load_state_dict(disc_optimizer)
        if disc_scheduler is not None and self.sched_d is not None:
            self.sched_d.load_state_dict(disc_scheduler)
