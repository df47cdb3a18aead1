"""Teacher training CLI — drop-in for the reference's ``src/train_teacher_gnn.py``
(flags :272-290, flow :291-535).  Same flags, printed lines and artefacts:
the best-validation teacher writes ``../saved-features/<ds>-<enc>_<mode>.pkl``
= {'features': h} and ``../saved-models/<ds>-<enc>_<mode>.pkl`` =
{'gnn': state_dict, 'predictor': state_dict} with torch.save (:446-452), which
main.py (and the reference's main.py) read.

Encoders: 'sage' (SAGEConv; SAGEConv_updated for coauthor-physics, :376-383)
and 'gcn' (:384-387) on llp_teacher.TeacherEngine, 'mlp' on the full-batch
engine.  Additive
flags: --dtype {fp32,bf16}, --synthetic (see main.py).
"""
import argparse
import os

import torch

import llp_datasets
import llp_split
import llp_train
from llp_sage import SAGEConv, SAGEConv_updated
from logger import Logger, ProductionLogger
from main import print_epoch, seed_everything, _write_summary
from models import GCN, MLP, SAGE, LinkPredictor


def build_parser():
    p = argparse.ArgumentParser(description='OGBL-DDI (GNN)')
    p.add_argument('--device', type=int, default=0)
    p.add_argument('--log_steps', type=int, default=1)
    p.add_argument('--encoder', type=str, default='sage')
    p.add_argument('--num_layers', type=int, default=2)
    p.add_argument('--hidden_channels', type=int, default=256)
    p.add_argument('--dropout', type=float, default=0.5)
    p.add_argument('--batch_size', type=int, default=64 * 1024)
    p.add_argument('--lr', type=float, default=0.005)
    p.add_argument('--epochs', type=int, default=20000)
    p.add_argument('--eval_steps', type=int, default=5)
    p.add_argument('--runs', type=int, default=5)
    p.add_argument('--dataset_dir', type=str, default='../data')
    p.add_argument('--datasets', type=str, default='cora')
    p.add_argument('--predictor', type=str, default='mlp', choices=['inner', 'mlp'])
    p.add_argument('--patience', type=int, default=100, help='number of patience steps for early stopping')
    p.add_argument('--metric', type=str, default='Hits@20', choices=['auc', 'hits@20', 'hits@50'],
                   help='main evaluation metric')
    p.add_argument('--use_valedges_as_input', action='store_true')
    p.add_argument('--transductive', type=str, default='transductive', choices=['transductive', 'production'])
    p.add_argument('--minibatch', action='store_true')
    # additive
    p.add_argument('--dtype', type=str, default='fp32', choices=['fp32', 'bf16'])
    p.add_argument('--synthetic', action='store_true')
    return p


def main(argv=None):
    args = build_parser().parse_args(argv)
    print(args)
    os.makedirs("../results", exist_ok=True)
    logger_file = "../results/" + args.datasets + "_supervised_" + args.transductive + ".txt"
    with open(logger_file, "a") as f:
        f.write(str(args))
        f.write(args.encoder + " as the encoder\n")
    if not torch.cuda.is_available():
        raise RuntimeError("the LLP trainer runs on an MI355X (HIP device) only — no CPU fallback")
    device = torch.device(f'cuda:{args.device}')
    torch.cuda.set_device(device)
    transductive = args.transductive == "transductive"
    if transductive:
        data, split_edge = llp_datasets.load_transductive(args.datasets, args.dataset_dir, args.synthetic)
        args.metric = 'Hits@50' if args.datasets == "collab" else 'Hits@20'
        data.x = data.x.to(device)
        input_size = data.x.size(1)
    else:
        # src/train_teacher_gnn.py:340-369: load the cached split or make it (seed 234)
        training_data, val_data, inference_data, _, test_edge_bundle, negative_samples = \
            llp_split.production_split(args.datasets, args.dataset_dir, args.synthetic)
        input_size = training_data.x.size(1)
        args.metric = 'Hits@20'
        training_data.to(device)
        val_data.to(device)
        inference_data.to(device)

    if args.encoder == 'sage':
        conv = SAGEConv_updated if args.datasets == "coauthor-physics" else SAGEConv
        model = SAGE(args.datasets, input_size, args.hidden_channels, args.hidden_channels, args.num_layers,
                     args.dropout, conv).to(device)
    elif args.encoder == 'gcn':
        model = GCN(input_size, args.hidden_channels, args.hidden_channels, args.num_layers, args.dropout).to(device)
    elif args.encoder == 'mlp':
        model = MLP(args.num_layers, input_size, args.hidden_channels, args.hidden_channels, args.dropout).to(device)
    else:
        raise ValueError(f"unknown encoder {args.encoder!r}")
    predictor = LinkPredictor(args.predictor, args.hidden_channels, args.hidden_channels, 1, 2,
                              args.dropout).to(device)

    if not transductive:
        loggers = {k: ProductionLogger(args.runs, args) for k in ('Hits@10', 'Hits@20', 'Hits@30', 'Hits@50', 'AUC')}
    else:
        Ks = ('Hits@10', 'Hits@50', 'Hits@100') if args.datasets == "collab" else \
            ('Hits@10', 'Hits@20', 'Hits@30', 'Hits@50')
        loggers = {k: Logger(args.runs, args) for k in Ks + ('AUC',)}
    tag = args.datasets + "-" + args.encoder + "_" + args.transductive + ".pkl"
    val_max = 0.0
    for run in range(args.runs):
        seed_everything(run)
        model.reset_parameters()
        predictor.reset_parameters()
        optimizer = torch.optim.Adam(list(model.parameters()) + list(predictor.parameters()), lr=args.lr)
        cnt_wait = 0
        best_val = 0.0
        for epoch in range(1, 1 + args.epochs):
            if transductive:
                loss = llp_train.train_teacher(model, predictor, data, split_edge, optimizer, args.batch_size,
                                               args.encoder, args.datasets, args.transductive, dtype=args.dtype)
                results, h = llp_train.test_transductive(model, predictor, data, split_edge, None, args.batch_size,
                                                         args.encoder, args.datasets, args)
            else:
                loss = llp_train.train_teacher(model, predictor, training_data, None, optimizer, args.batch_size,
                                               args.encoder, args.datasets, args.transductive, dtype=args.dtype)
                results, h = llp_train.test_production(model, predictor, val_data, inference_data,
                                                       test_edge_bundle, negative_samples, None, args.batch_size,
                                                       args.encoder, args.datasets)
            if results[args.metric][0] > val_max:
                val_max = results[args.metric][0]
                if args.encoder != 'mlp':
                    os.makedirs("../saved-features", exist_ok=True)
                    os.makedirs("../saved-models", exist_ok=True)
                    torch.save({'features': h}, "../saved-features/" + tag)
                    torch.save({'gnn': model.state_dict(), 'predictor': predictor.state_dict()},
                               "../saved-models/" + tag)
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
