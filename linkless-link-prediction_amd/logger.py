"""Result loggers with the reference's interface and printed output
(src/logger.py:3-89): ``Logger`` keeps (valid, test) pairs per epoch,
``ProductionLogger`` keeps (val, test, old_old, old_new, new_new).

``print_statistics(run)`` reports the epoch with the best first column;
``print_statistics()`` reports mean ± std over runs of 100 x the best-epoch
values, in the reference's exact line formats.
"""
import torch


class _RunTable:
    width = 2

    def __init__(self, runs, info=None):
        self.info = info
        self.results = [[] for _ in range(runs)]

    def add_result(self, run, result):
        assert len(result) == self.width
        assert 0 <= run < len(self.results)
        self.results[run].append(result)

    def reset(self, run):
        assert 0 <= run < len(self.results)
        self.results[run] = []

    def _best_rows(self):
        """Per run: the row (x100) of the epoch with the highest first column."""
        rows = []
        for r in self.results:
            t = 100 * torch.tensor(r)
            rows.append(t[t[:, 0].argmax()])
        return torch.stack(rows)


class Logger(_RunTable):
    """Transductive setting: overall result only."""
    width = 2

    def print_statistics(self, run=None):
        if run is not None:
            t = torch.tensor(self.results[run])
            best = t[:, 0].argmax().item()
            print(f'Run {run + 1:02d}:')
            print(f'Highest Valid: {t[:, 0].max():.4f}')
            print(f'   Final Test: {t[best, 1]:.4f}')
            return
        per_run = []
        for r in self.results:
            t = 100 * torch.tensor(r)
            per_run.append((t[:, 0].max().item(), t[t[:, 0].argmax(), 1].item()))
        b = torch.tensor(per_run)
        print('All runs:')
        print(f'Highest Valid: {b[:, 0].mean():.2f} ± {b[:, 0].std():.2f}')
        print(f'   Final Test: {b[:, 1].mean():.2f} ± {b[:, 1].std():.2f}')


class ProductionLogger(_RunTable):
    """Production setting: old_old / old_new / new_new reported separately."""
    width = 5
    _labels = ('  Final val', '   Final Test', '   old_old Test', '   old_new Test', '   new_new Test')
    _labels_all = ('  Final val', '   Final Test', '   Final old_old', '   Final old_new', '   Final new_new')

    def print_statistics(self, run=None):
        if run is not None:
            t = 100 * torch.tensor(self.results[run])
            row = t[t[:, 0].argmax()]
            print(f'Run {run + 1:02d}:')
            for label, v in zip(self._labels, row.tolist()):
                print(f'{label}: {v:.2f}')
            return
        b = self._best_rows()
        print('All runs:')
        for i, label in enumerate(self._labels_all):
            print(f'{label}: {b[:, i].mean():.2f} ± {b[:, i].std():.2f}')
