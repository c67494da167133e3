"""Training CLI — drop-in for the reference's train.py (flags train.py:26-77, loop 84-334).

    python train.py [--batch_size=20] [--learning_rate=1e-3] [--train_range=REFINE|ALL] ...
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 train.py ...

Same flag names and defaults as the reference, plus: --train_range (the reference
hard-codes REFINE at train.py:130), --img_height/--img_width (config.img_size), --dtype
(fp32 like the reference's DTYPE, or bf16), --dataset_dir, --seed.  Data parallel when
launched with several ranks (RCCL all-reduce of the flat gradient, global-batch loss
normalisation; --batch_size is then per GPU).  Checkpoints are torch files holding the
slim-named variables and global_step.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

import config  # noqa: E402
from utils.common_tools import logger  # noqa: E402


def str2bool(v):
    if isinstance(v, bool):
        return v
    return str(v).lower() in ('1', 'true', 't', 'yes', 'y')


def none_or_str(v):
    return None if v in (None, '', 'None', 'none') else v


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument('--backbone_name', default='mobilenet_v2')
    ap.add_argument('--learning_rate', type=float, default=1e-3)
    ap.add_argument('--batch_size', type=int, default=20)
    ap.add_argument('--num_readers', type=int, default=4)
    ap.add_argument('--num_preprocessing_threads', type=int, default=4)
    ap.add_argument('--checkpoint_all', type=none_or_str, default=None)
    ap.add_argument('--checkpoint_refine', type=none_or_str, default='checkpoint/mbn_none53x35/refine/mobilenet_v2.model')
    ap.add_argument('--train_dir', default='checkpoint/')
    ap.add_argument('--summary_dir', default='summary/')
    ap.add_argument('--max_number_of_steps', type=int, default=None)
    ap.add_argument('--log_every_n_steps', type=int, default=20)
    ap.add_argument('--summary_every_n_steps', type=int, default=20)
    ap.add_argument('--save_every_n_steps', type=int, default=2000)
    ap.add_argument('--fix_refine', type=str2bool, default=True)
    # additions
    ap.add_argument('--sync_bn', type=str2bool, default=False,
                    help='data parallel: BatchNorm statistics over the global batch (default per rank; '
                         'the reference runs on one device)')
    ap.add_argument('--train_range', default='REFINE', choices=['REFINE', 'ALL'])
    ap.add_argument('--img_height', type=int, default=config.img_size[0])
    ap.add_argument('--img_width', type=int, default=config.img_size[1])
    ap.add_argument('--dtype', default='fp32', choices=['fp32', 'bf16'])
    ap.add_argument('--dataset_dir', default='./dataset/bdd100k_TfRecord/')
    ap.add_argument('--synthetic', type=str2bool, default=False,
                    help='run on synthetic BDD-shaped batches (no dataset needed); results are not real '
                         'metrics.  Without it a missing dataset or checkpoint is an error')
    ap.add_argument('--seed', type=int, default=0)
    ap.add_argument('--save_format', default='torch', choices=['torch', 'tf'],
                    help='checkpoint format: torch file, or a TF-1.x tensor bundle the reference can restore')
    ap.add_argument('--augment', type=str2bool, default=True,
                    help='process_raw_data_train on the GPU (random crop / flip / colour); False = raw batches')
    ap.add_argument('--hip_graph', type=str2bool, default=True,
                    help='replay the training step as a HIP graph (Trainer.step_graphed, bit-identical to the '
                         'eager step; dropout steps run eager).  Data parallel over RCCL: the whole step, its '
                         'collectives included (the library\'s communicator; gradient buckets on a side stream)')
    return ap.parse_args(argv)


def load_ckpt(store, path, names_regex=None):
    """saver.restore (train.py:188, 282) / restore_saver of backbone.+|refine.+ (155-158, 191-193):
    a torch checkpoint written by this CLI or a TF-1.x tensor bundle of the reference."""
    from rod.checkpoint import load_variables
    return load_variables(store, path, names_regex=names_regex)


def save_ckpt(store, path, step, fmt='torch'):
    from rod.checkpoint import save_variables
    save_variables(store, path, step, fmt)


def _loss_copy(losses, world):
    """The step's loss values as one small device tensor (a copy: a replayed graph overwrites
    its outputs on the next replay).  Data parallel: each rank holds its shard's sum / global
    batch, so the global loss is the all-reduced sum."""
    lv = torch.stack([l.detach().float().reshape(()) for l in losses])
    if world > 1:
        torch.distributed.all_reduce(lv)
    if lv.device.type != 'cuda':
        return lv, None
    host = torch.empty(lv.shape, dtype=lv.dtype, pin_memory=True)
    host.copy_(lv, non_blocking=True)   # queued before the next step: reading it waits for this step only
    ev = torch.cuda.Event()
    ev.record()
    return host, ev


def _loss_values(entry):
    host, ev = entry
    if ev is not None:
        ev.synchronize()
    return host.tolist()


class StepLog(object):
    """Running averages and the log / summary lines of train.py:292-320 (formats kept)."""

    def __init__(self, F, trainer, tr_range, rank, summ):
        self.F, self.trainer, self.tr_range, self.rank, self.summ = F, trainer, tr_range, rank, summ
        self.avg = [0., 0., 0.]
        self.avg_t = 0.

    def __call__(self, current_step, vals, t):
        F, avg = self.F, self.avg
        if F.log_every_n_steps is not None:
            s = current_step % F.log_every_n_steps
            if self.tr_range is config.train_range.ALL:
                tot, _, dl, cl = vals
                avg[:] = [(avg[0] * s + tot) / (s + 1.), (avg[1] * s + dl) / (s + 1.), (avg[2] * s + cl) / (s + 1.)]
            else:
                avg[0] = (avg[0] * s + vals[0]) / (s + 1.)
            self.avg_t = (self.avg_t * s + t) / (s + 1.)
            if current_step % F.log_every_n_steps == F.log_every_n_steps - 1 and self.rank == 0:
                if self.tr_range is config.train_range.ALL:
                    logger.info('Step%s total_loss:%s det_loss:%s clf_loss:%s time_each_step:%s' %
                                (str(current_step + 1), str(avg[0]), str(avg[1]), str(avg[2]), str(self.avg_t)))
                else:
                    logger.info('Step_%s refine_loss:%s time:%s' % (str(current_step + 1), str(avg[0]),
                                                                    str(self.avg_t)))
                avg[:] = [0., 0., 0.]
                self.avg_t = 0.
        if self.summ is not None and F.summary_every_n_steps is not None and \
                current_step % F.summary_every_n_steps == F.summary_every_n_steps - 1:
            rec = {'step': current_step, 'loss': vals, 'lr': self.trainer.opt.decayed_lr(current_step)}
            self.summ.write(json.dumps(rec) + '\n')
            self.summ.flush()


def main(argv=None):
    F = parse(argv)
    logger.info('Asserting parameters')
    assert F.batch_size > 0
    assert F.learning_rate >= 0.
    assert F.log_every_n_steps is None or F.log_every_n_steps > 0
    assert F.summary_every_n_steps is None or F.summary_every_n_steps > 0
    assert F.save_every_n_steps is None or F.save_every_n_steps > 0
    assert F.backbone_name in config.supported_backbone_name

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        torch.cuda.set_device(local)
        torch.distributed.init_process_group('nccl', device_id=torch.device('cuda', local))
    dev = torch.device('cuda', local)
    from rod.dataio import make_source
    from rod.ddp import make_reducer
    from rod.trainer import Trainer

    config.img_size = (F.img_height, F.img_width)
    tr_range = getattr(config.train_range, F.train_range)
    dtype = torch.bfloat16 if F.dtype == 'bf16' else torch.float32
    logger.info('Building model, using backbone---%s' % F.backbone_name)
    trainer = Trainer(config.img_size, F.batch_size, dtype=dtype, train_range=tr_range, learning_rate=F.learning_rate,
                      device=dev, fix_refine=F.fix_refine, seed=F.seed, world_size=world,
                      reducer=make_reducer(world, rank) if world > 1 else None, backbone_name=F.backbone_name,
                      sync_bn=F.sync_bn)
    store = trainer.net.store
    logger.info('Total trainable parameters:%s' % str(store.trainable_count()))
    step0 = 0
    if tr_range is config.train_range.ALL:
        if F.checkpoint_all is not None:
            step0 = load_ckpt(store, F.checkpoint_all)
            logger.info('Load checkpoint for all net success...')
        if F.checkpoint_refine is not None:
            load_ckpt(store, F.checkpoint_refine, names_regex=r'backbone.+|refine.+')
            logger.info('Load checkpoint for refine net success...')
    else:
        if F.checkpoint_refine is not None:
            step0 = load_ckpt(store, F.checkpoint_refine)
            logger.info('Load checkpoint success...')
        else:
            logger.info('TF variables init success...')
    trainer.opt.global_step = step0
    logger.info('Building data pileline, using dataset---%s' % 'bdd100k_train')
    source = make_source(F.dataset_dir, F.batch_size, config.img_size, dev, seed=F.seed,
                         augment_dtype=dtype if F.augment else None, synthetic=F.synthetic, dtype=dtype,
                         num_readers=F.num_readers, rank=rank, world=world)

    os.makedirs(F.summary_dir, exist_ok=True)
    summ = open(os.path.join(F.summary_dir, 'train_rank%d.jsonl' % rank), 'a') if rank == 0 else None
    log = StepLog(F, trainer, tr_range, rank, summ)
    # Trainer.graph_mode: the whole step as one graph (one process, or data parallel through the
    # library's RCCL communicator), forward + backward only (gloo), or eager (dropout)
    step = trainer.step_graphed if F.hip_graph else trainer.step
    # the host reads each step's losses (the reference's sess.run returns them) one step late:
    # step k+1 is queued on the GPU before step k's values are read, so the GPU does not wait
    # for the host's logging and next-batch work.  Checkpoints are written right after their
    # step (before the next is queued), so they hold exactly that step's parameters.
    pending = None
    last = time.time()
    while True:
        losses = step(*next(source))
        current_step = trainer.opt.global_step - 1
        entry = (current_step, _loss_copy(losses, world))
        if F.save_every_n_steps is not None and current_step % F.save_every_n_steps == F.save_every_n_steps - 1 \
                and rank == 0:
            logger.info('Saving model...')
            save_ckpt(store, os.path.join(F.train_dir, F.backbone_name + '.model'), current_step + 1, F.save_format)
            logger.info('Save model sucess...')
        if pending is not None:
            vals = _loss_values(pending[1])   # waits for the previous step only
            now = time.time()
            log(pending[0], vals, round(now - last, 3))
            last = now
        pending = entry
        if F.max_number_of_steps is not None and current_step >= F.max_number_of_steps:
            break
    vals = _loss_values(pending[1])
    log(pending[0], vals, round(time.time() - last, 3))
    logger.info('Exit training...')
    close = getattr(source, 'close', None)
    if close is not None:
        close()
    if world > 1:
        if getattr(trainer.reducer, 'native', False):
            from rod import _abi
            _abi.call('rod_rccl_destroy')
        torch.distributed.destroy_process_group()


if __name__ == '__main__':
    main()
