"""train.py drop-in (train.py:1-244 of the reference) on MI355X.

Same positional arguments (CKPT_PATH_PFX ARCH_FILE PAR_FILE SAMPLES_FILE) and flags; the
TF session/graph becomes WaveNetTrain's lbwn plan, the optimizer lbwn's TF1 Adam, the
dataset MaskedSliceWav.  Checkpoints: '<pfx>.net-<step>.safetensors' (model variables under
the reference serial names + Adam slots) and '<pfx>.dset-<step>.safetensors' (shuffle seed
and file position), at the reference's cadence (train.py:236-240).

Multi-GPU: launch with torch.distributed.run (one process per GPU); --batch-size is then
the per-GPU batch, the dealer runs over the global batch and each rank trains on its rows,
gradients are summed over ranks before the (replicated) Adam step (lbwn.dist).

TF-only switches are accepted for command-line compatibility: --tf-eager is implied,
--add-summary/--tb-dir/--prof-dir/--timeline-file print what replaces them (rocprofv3),
--tf-debug and --cpu-only exit(1) (there is no CPU execution path).
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)


def get_args(argv=None):
    p = argparse.ArgumentParser(description='WaveNet')
    p.add_argument('--timeline-file', '-tf', type=str, help='Enable profiling and write info to <timeline_file>')
    p.add_argument('--prof-dir', '-pd', type=str, metavar='DIR', help='Output profiling events to <prof_dir>')
    p.add_argument('--resume-step', '-rs', type=int, metavar='INT',
                   help='Resume training from CKPT_DIR/<ckpt_pfx>-<resume_step> checkpoints')
    p.add_argument('--add-summary', '-s', action='store_true', default=False,
                   help='If present, add summary histogram nodes to graph for TensorBoard')
    p.add_argument('--cpu-only', '-cpu', action='store_true', default=False,
                   help='If present, do all computation on CPU')
    p.add_argument('--tb-dir', '-tb', type=str, metavar='DIR', help='TensorBoard directory for summary events')
    p.add_argument('--save-interval', '-si', type=int, default=1000, metavar='INT',
                   help='Save a checkpoint after this many steps each time')
    p.add_argument('--progress-interval', '-pi', type=int, default=10, metavar='INT',
                   help='Print a progress message at this interval')
    p.add_argument('--tf-debug', '-tdb', action='store_true', default=False, help='Enable tf_debug debugging console')
    p.add_argument('--tf-eager', '-te', action='store_true', default=False, help='Enable tf Eager mode')
    p.add_argument('--max-steps', '-ms', type=int, default=int(1e20), help='Maximum number of training steps')
    p.add_argument('--batch-size', '-bs', type=int, metavar='INT', help='Batch size (overrides PAR_FILE setting)')
    p.add_argument('--slice-size', '-ss', type=int, metavar='INT', help='Slice size (overrides PAR_FILE setting)')
    p.add_argument('--l2-factor', '-l2', type=float, metavar='FLOAT', help='Loss = Xent loss + l2_factor * l2_loss')
    p.add_argument('--learning-rate', '-lr', type=float, metavar='FLOAT',
                   help='Learning rate (overrides PAR_FILE setting)')
    p.add_argument('--num-global-cond', '-gc', type=int, metavar='INT',
                   help='Number of global conditioning categories')
    p.add_argument('--seed', type=int, default=None, help='(build extension) weight / shuffle seed')
    p.add_argument('ckpt_path', type=str, metavar='CKPT_PATH_PFX')
    p.add_argument('arch_file', type=str, metavar='ARCH_FILE')
    p.add_argument('par_file', type=str, metavar='PAR_FILE')
    p.add_argument('sam_file', type=str, metavar='SAMPLES_FILE')
    return p.parse_args(argv)


def prepare_arch(arch, num_global_cond):
    """The ARCH_FILE dict brought to WaveNetTrain's 14 keys; -gc may supply the
    n_gc_category the file lacks (train.py:77-80, :138-146: par/arch2.json, arch4.json).
    Errors print to stderr and exit(1), like the reference."""
    from lbwn.arch import ArchError, normalize_arch
    try:
        return normalize_arch(arch, num_global_cond=num_global_cond)
    except ArchError as e:
        print(str(e), file=sys.stderr)
        sys.exit(1)


def main(argv=None):
    args = get_args(argv)
    from sys import stderr

    with open(args.arch_file) as fp:
        arch = json.load(fp)
    with open(args.par_file) as fp:
        par = json.load(fp)

    if args.num_global_cond is None and 'n_gc_category' not in arch:     # train.py:77-80
        print('Error: must provide n_gc_category in ARCH_FILE, or --num-global-cond', file=stderr)
        sys.exit(1)
    if args.tf_eager and args.tf_debug:
        print('Error: --tf-debug and --tf-eager cannot both be set', file=stderr)
        sys.exit(1)
    if args.tf_debug or args.cpu_only:
        print('Error: --tf-debug / --cpu-only have no equivalent here: the training step runs only as '
              'HIP kernels on an MI355X (liblbwn.so)', file=stderr)
        sys.exit(1)
    if args.add_summary and args.tb_dir is None:                           # train.py:206-210
        print('Error: must provide --tb-dir argument if there are summaries in the graph', file=stderr)
        sys.exit(1)
    for flag in ('timeline_file', 'prof_dir', 'tb_dir'):
        if getattr(args, flag):
            print('Note: --{} is a TF profiler/summary hook; profile this build with '
                  '`rocprofv3 --kernel-trace --stats -- python train.py ...`'.format(flag.replace('_', '-')),
                  file=stderr)

    if args.batch_size is not None:
        par['batch_sz'] = args.batch_size
    if args.slice_size is not None:
        par['slice_sz'] = args.slice_size
    if args.l2_factor is not None:
        par['l2_factor'] = args.l2_factor
    if args.learning_rate is not None:
        par['learning_rate'] = args.learning_rate

    import torch
    from lbwn import dist as lbdist
    from lbwn.arch import normalize_arch, mel_hop_sz as hop_of
    from lbwn.data import DeviceBatches, MaskedSliceWav
    from lbwn.optim import AdamOptimizer
    from lbwn.tmodel import WaveNetTrain

    arch = prepare_arch(arch, args.num_global_cond)
    dp = lbdist.init()
    hop = hop_of(arch)
    B = par['batch_sz']
    dset = MaskedSliceWav(None, args.sam_file, par['sample_rate'], par['slice_sz'], par['prefetch_sz'],
                          arch['n_lc_in'], hop, B * dp.world, par['n_keep_checkpoints'],
                          '{}.dset'.format(args.ckpt_path), args.resume_step or 0, random_seed=args.seed,
                          rows=dp.rows(B) if dp.enabled else None)
    dset.init_sample_catalog()
    if args.num_global_cond is not None:                                    # train.py:138-145
        if args.num_global_cond < dset.get_max_id():
            print('Error: --num-global-cond must be >= {}, the highest ID in the dataset.'.format(
                dset.get_max_id()), file=stderr)
            sys.exit(1)
        arch['n_gc_category'] = args.num_global_cond
        arch = normalize_arch(arch)

    net = WaveNetTrain(**arch, batch_sz=B, l2_factor=par['l2_factor'], add_summary=par.get('add_summary', False),
                       n_keep_checkpoints=par['n_keep_checkpoints'], ckpt_path='{}.net'.format(args.ckpt_path),
                       resume_step=args.resume_step or 0, n_valid_total=par.get('n_valid_total', 0),
                       print_interval=args.progress_interval if dp.rank == 0 else 0,
                       seed=args.seed if args.seed is not None else 0)
    net.dp = dp
    dset.set_receptive_field_size(net.get_recep_field_sz())
    dset.build()
    dset.init_vars()
    optimizer = AdamOptimizer(learning_rate=par['learning_rate'])
    print('Built graph.', file=stderr)

    if args.resume_step:
        net.restore(optimizer)
        dset.restore()
        print('Restored net and dset from checkpoint', file=stderr)
    dp.broadcast_params(net)

    print('Starting training...', file=stderr)
    step = args.resume_step or 1
    itr = DeviceBatches(dset.get_itr(), net.device)   # pinned buffers, non-blocking H2D: no per-step sync
    while step < args.max_steps:
        try:
            file_read_count, wav_input, mel_input, id_mask = next(itr)
        except StopIteration:
            break
        net.forward(wav_input, mel_input, id_mask, backward=True)
        dp.reduce_grads(net)
        if args.progress_interval and net.global_step_host % args.progress_interval == 0:
            net.check_status()                # cumulative: any timed-out step since the start (never applied)
        net.maybe_print()                     # tmodel.py:272-281 prints before the step counters advance
        optimizer.apply(net)
        if step % args.save_interval == 0 and step != args.resume_step:
            net.check_status()
            net_save_path = net.save(step, optimizer)        # collective under DP
            if dp.rank == 0:
                dset_save_path = dset.save(step, file_read_count)
                print('Saved checkpoints to {} and {}'.format(net_save_path, dset_save_path), file=stderr)
        step += 1
    torch.cuda.synchronize()
    if step > (args.resume_step or 1):
        net.check_status()
    return net


if __name__ == '__main__':
    main()
