"""LLP student distillation CLI — drop-in for the reference's ``src/main.py``
(flags src/main.py:240-269, flow :296-513, printed lines :437-456, results
file :465-513).  Same flags and outputs; additive flags only:

  --dtype {fp32,bf16}   compute dtype of the HIP engine (fp32 = the reference's)
  --synthetic           seeded graph of the dataset's shape when no dataset
                        file exists (no network here; see llp_datasets.py)

Training runs in llp_train (DistillEngine, hand-written gfx950 kernels);
evaluation in llp_eval (device Hits@K / AUC).  Teacher artefacts are read
from ``../saved-models/<ds>-<enc>_<mode>.pkl`` and
``../saved-features/<ds>-<enc>_<mode>.pkl`` exactly as the reference does
(src/main.py:356-363), with ``torch.load(weights_only=True)``.
"""
import argparse
import os
import random

import numpy as np
import torch

import llp_datasets
import llp_split
import llp_train
from logger import Logger, ProductionLogger
from models import MLP, LinkPredictor


def seed_everything(seed):
    """torch_geometric.seed.seed_everything (src/main.py:397)."""
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    torch.cuda.manual_seed_all(seed)


def build_parser():
    p = argparse.ArgumentParser(description='OGBL-DDI (GNN)')
    p.add_argument('--device', type=int, default=0)
    p.add_argument('--log_steps', type=int, default=1)
    p.add_argument('--encoder', type=str, default='sage')
    p.add_argument('--num_layers', type=int, default=2)
    p.add_argument('--hidden_channels', type=int, default=256)
    p.add_argument('--dropout', type=float, default=0.5)
    p.add_argument('--link_batch_size', type=int, default=64 * 1024)
    p.add_argument('--node_batch_size', type=int, default=64 * 1024)
    p.add_argument('--lr', type=float, default=0.005)
    p.add_argument('--epochs', type=int, default=20000)
    p.add_argument('--eval_steps', type=int, default=5)
    p.add_argument('--runs', type=int, default=10)
    p.add_argument('--dataset_dir', type=str, default='../data')
    p.add_argument('--datasets', type=str, default='collab')
    p.add_argument('--predictor', type=str, default='mlp', choices=['inner', 'mlp'])
    p.add_argument('--patience', type=int, default=100, help='number of patience steps for early stopping')
    p.add_argument('--metric', type=str, default='Hits@20', choices=['auc', 'hits@20', 'hits@50'],
                   help='main evaluation metric')
    p.add_argument('--use_valedges_as_input', action='store_true')
    p.add_argument('--True_label', default=0.1, type=float, help="true_label loss")
    p.add_argument('--KD_RM', default=0, type=float, help="Representation-based matching KD")
    p.add_argument('--KD_LM', default=0, type=float, help="logit-based matching KD")
    p.add_argument('--LLP_D', default=1, type=float, help="distribution-based matching kd")
    p.add_argument('--LLP_R', default=1, type=float, help="rank-based matching kd")
    p.add_argument('--margin', default=0.1, type=float, help="margin for rank-based kd")
    p.add_argument('--rw_step', type=int, default=3, help="nearby nodes sampled times")
    p.add_argument('--ns_rate', type=int, default=1, help="randomly sampled rate over # nearby nodes")
    p.add_argument('--hops', type=int, default=2, help="random_walk step for each sampling time")
    p.add_argument('--ps_method', type=str, default='nb', help="positive sampling is rw or nb")
    p.add_argument('--transductive', type=str, default='transductive', choices=['transductive', 'production'])
    p.add_argument('--minibatch', action='store_true')
    # additive
    p.add_argument('--dtype', type=str, default='fp32', choices=['fp32', 'bf16'])
    p.add_argument('--synthetic', action='store_true')
    return p


def _results_header(args):
    if args.KD_RM != 0:
        return "Logit-matching\n"
    if args.KD_LM != 0:
        return "Representation-matching\n"
    if args.LLP_D != 0 or args.LLP_R != 0:
        return "LLP (Relational Distillation)\n"
    return ""


def _write_summary(path, loggers, transductive):
    with open(path, "a") as f:
        f.write('All runs:\n')
        for key, lg in loggers.items():
            print(key)
            lg.print_statistics()
            f.write(f'{key}:\n')
            if transductive:
                best = []
                for r in lg.results:
                    r = 100 * torch.tensor(r)
                    best.append((r[:, 0].max().item(), r[r[:, 0].argmax(), 1].item()))
                r = torch.tensor(best)[:, 1]
                f.write(f'Test: {r.mean():.4f} ± {r.std():.4f}\n')
            else:
                best = []
                for r in lg.results:
                    r = 100 * torch.tensor(r)
                    best.append(tuple(r[r[:, 0].argmax(), i].item() for i in range(5)))
                b = torch.tensor(best)
                names = ('  Final val', '   Final Test', '   Final old_old', '   Final old_new', '   Final new_new')
                for i, n in enumerate(names):
                    f.write(f'{n}: {b[:, i].mean():.2f} ± {b[:, i].std():.2f}' + ('\n' if i == 4 else ''))


def print_epoch(results, run, epoch, loss, transductive):
    """Per-epoch lines of src/main.py:435-456 (train_teacher_gnn.py:463-487)."""
    for key, result in results.items():
        print(key)
        if transductive:
            valid_hits, test_hits = result
            print(f'Run: {run + 1:02d}, '
                  f'Epoch: {epoch:02d}, '
                  f'Loss: {loss:.4f}, '
                  f'Valid: {100 * valid_hits:.2f}%, '
                  f'Test: {100 * test_hits:.2f}%')
        else:
            valid_hits, test_hits, old_old, old_new, new_new = result
            print(f'Run: {run + 1:02d}, '
                  f'Epoch: {epoch:02d}, '
                  f'Loss: {loss:.4f}, '
                  f'valid: {100 * valid_hits:.2f}%, '
                  f'test: {100 * test_hits:.2f}%, '
                  f'old_old: {100 * old_old:.2f}%, '
                  f'old_new: {100 * old_new:.2f}%, '
                  f'new_new: {100 * new_new:.2f}%')
    print('---')


def main(argv=None):
    args = build_parser().parse_args(argv)
    print(args)
    os.makedirs("../results", exist_ok=True)
    logger_file = "../results/" + args.datasets + "_KD_" + args.transductive + ".txt"
    with open(logger_file, "a") as f:
        f.write(str(args) + "\n")
        f.write(_results_header(args))

    if not torch.cuda.is_available():
        raise RuntimeError("the LLP trainer runs on an MI355X (HIP device) only — no CPU fallback")
    device = torch.device(f'cuda:{args.device}')
    torch.cuda.set_device(device)

    transductive = args.transductive == "transductive"
    if transductive:
        data, split_edge = llp_datasets.load_transductive(args.datasets, args.dataset_dir, args.synthetic)
        args.metric = 'Hits@50' if args.datasets == "collab" else 'Hits@20'
        input_size = data.x.size(1)
        if not args.minibatch:
            data.x = data.x.to(device)
        args.node_batch_size = int(data.x.size(0) / (split_edge['train']['edge'].size(0) / args.link_batch_size))
    else:
        # src/main.py:337-346: the split train_teacher_gnn.py cached (made here when absent)
        training_data, val_data, inference_data, data, test_edge_bundle, negative_samples = \
            llp_split.production_split(args.datasets, args.dataset_dir, args.synthetic)
        input_size = training_data.x.size(1)
        if not args.minibatch:
            training_data.to(device)
        val_data.to(device)
        inference_data.to(device)
        args.node_batch_size = int(training_data.x.size(0) /
                                   (training_data.edge_index.size(1) / args.link_batch_size))

    model = MLP(args.num_layers, input_size, args.hidden_channels, args.hidden_channels, args.dropout).to(device)
    predictor = LinkPredictor(args.predictor, args.hidden_channels, args.hidden_channels, 1, args.num_layers,
                              args.dropout).to(device)
    tag = args.datasets + "-" + args.encoder + "_" + args.transductive + ".pkl"
    pretrained = torch.load("../saved-models/" + tag, weights_only=True, map_location="cpu")
    teacher_predictor = LinkPredictor(args.predictor, 256, 256, 1, 2, args.dropout)
    teacher_predictor.load_state_dict(pretrained['predictor'], strict=True)
    teacher_predictor.to(device)
    t_h = torch.load("../saved-features/" + tag, weights_only=True, map_location="cpu")['features']
    for p in teacher_predictor.parameters():
        p.requires_grad = False

    if not transductive:
        loggers = {k: ProductionLogger(args.runs, args) for k in ('Hits@10', 'Hits@20', 'Hits@30', 'Hits@50', 'AUC')}
    else:
        Ks = ('Hits@10', 'Hits@50', 'Hits@100') if args.datasets == "collab" else \
            ('Hits@10', 'Hits@20', 'Hits@30', 'Hits@50')
        loggers = {k: Logger(args.runs, args) for k in Ks + ('AUC',)}

    for run in range(args.runs):
        seed_everything(run + 1)
        model.reset_parameters()
        predictor.reset_parameters()
        optimizer = torch.optim.Adam(list(model.parameters()) + list(predictor.parameters()), lr=args.lr)
        cnt_wait = 0
        best_val = 0.0
        for epoch in range(1, 1 + args.epochs):
            if transductive:
                fn = llp_train.train_minibatch if args.minibatch else llp_train.train
                loss = fn(model, predictor, t_h, teacher_predictor, data, split_edge, optimizer, args, device)
                results, h = llp_train.test_transductive(model, predictor, data, split_edge, None,
                                                         args.link_batch_size, 'mlp', args.datasets, args)
            else:   # src/main.py:420-423: full-batch train() in the production setting
                loss = llp_train.train(model, predictor, t_h, teacher_predictor, training_data, None, optimizer,
                                       args, device)
                results, h = llp_train.test_production(model, predictor, val_data, inference_data,
                                                       test_edge_bundle, negative_samples, None,
                                                       args.link_batch_size, 'mlp', args.datasets)
            if results[args.metric][0] >= best_val:
                best_val = results[args.metric][0]
                cnt_wait = 0
            else:
                cnt_wait += 1
            for key, result in results.items():
                loggers[key].add_result(run, result)
            if epoch % args.log_steps == 0:
                print_epoch(results, run, epoch, loss, transductive)
            if cnt_wait >= args.patience:
                break
        for key in loggers.keys():
            print(key)
            loggers[key].print_statistics(run)

    _write_summary(logger_file, loggers, transductive)


if __name__ == "__main__":
    main()
