"""Summarise an SGPU_TIMELINE=1 stderr log: per-ticket phase durations."""
import collections
import sys

ev = collections.defaultdict(dict)
walls = []
for ln in open(sys.argv[1]):
    p = ln.split()
    if p and p[0] == 'eng':
        t = float(p[1])
        ticket = int(p[-1][1:])
        what = ' '.join(p[3:-1])
        ev[ticket].setdefault(what, t)
    elif p and p[0] == 'wall':
        walls.append(ln.strip())
tickets = sorted(ev)
# keep the second (timed) run: tickets after the largest gap
print(walls)
print('tickets', len(tickets))


def span(a, b):
    v = [ev[k][b] - ev[k][a] for k in tickets if a in ev[k] and b in ev[k]]
    return len(v), (sum(v) / len(v) * 1e3 if v else 0)


for a, b in [('enqueue', 'assembled'), ('enqueue', 'launch begin'), ('launch begin', 'launch end'),
             ('launch end', 'fence passed'), ('inline', 'fence passed'), ('enqueue', 'fence passed'),
             ('fence passed', 'complete end'), ('enqueue', 'complete end'), ('complete begin', 'fence passed')]:
    n, us = span(a, b)
    print('%-14s -> %-14s n=%6d mean %8.1f us' % (a, b, n, us))
starts = [ev[k]['enqueue'] for k in tickets if 'enqueue' in ev[k]]
if len(starts) > 1:
    gaps = [(starts[i + 1] - starts[i]) * 1e3 for i in range(len(starts) - 1)]
    gaps.sort()
    print('enqueue gap us: median %.1f p90 %.1f' % (gaps[len(gaps) // 2], gaps[int(len(gaps) * .9)]))
inl = sum(1 for k in tickets if 'inline' in ev[k])
print('inline tickets', inl)
