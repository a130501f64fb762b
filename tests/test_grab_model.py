"""CPU model of the fused kernel's work distribution (rt_path.h grab_chunk: partitioned
chunk counters, interleaved granules, the probe-and-move search with its `dead` mask).
Waves are interleaved at random and half of the probes read stale (low) counter values;
every chunk must be handed out exactly once and the search must end within NP + 1
atomics per refill.  CPU only: this pins the protocol, the GPU tests pin the kernel."""
import random

import pytest


def run(n_chunks, lg, gl, grab_min, n_waves, seed):
    rnd = random.Random(seed)
    NP = 1 << lg; G = 1 << gl
    granules = (n_chunks + G - 1) >> gl
    def part_end(p):
        return (((granules - p - 1) >> lg) + 1) << gl if granules > p else 0
    def chunk(p, pos):
        return ((((pos >> gl) << lg) + p) << gl) | (pos & (G - 1))
    ctr = [0] * 64
    stale = [0] * 64
    waves = [dict(next=0, end=0, part=w % NP, dead=0, need=rnd.randint(1, 64)) for w in range(n_waves)]
    got = []
    steps = 0
    active = list(range(n_waves))
    while active:
        steps += 1
        assert steps < 10**7
        wi = rnd.choice(active)
        b = waves[wi]
        n = b['need']
        avail = b['end'] - b['next']
        out = []
        if n <= avail:
            out = [(b['part'], b['next'] + r) for r in range(n)]
            b['next'] += n
        else:
            old_next, old_part = b['next'], b['part']
            g = gend = 0
            passes = 0
            while b['part'] < 64:
                passes += 1
                assert passes <= NP + 1
                endp = part_end(b['part'])
                want = max(grab_min, n - avail)
                g = ctr[b['part']]; ctr[b['part']] += want
                if rnd.random() < 0.5: stale[b['part']] = ctr[b['part']]
                if g < endp:
                    gend = min(g + want, endp); break
                b['dead'] |= 1 << b['part']
                live = 0
                for i in range(NP):
                    v = stale[i] if rnd.random() < 0.5 else ctr[i]
                    if v < part_end(i): live |= 1 << i
                live &= ~b['dead']
                if not live:
                    b['part'] = 64; break
                sh = b['part'] + 1
                rot = live if sh >= 64 else ((live >> sh) | (live << (64 - sh))) & (2**64 - 1)
                ffs = (rot & -rot).bit_length() - 1
                b['part'] = (sh + ffs) & 63
            for r in range(n):
                if r < avail:
                    out.append((old_part, old_next + r))
                else:
                    take = r - avail
                    if b['part'] >= 64 or g + take >= gend: continue
                    out.append((b['part'], g + take))
            b['next'] = min(g + (n - avail), gend); b['end'] = gend
        for p, pos in out:
            c = chunk(p, pos)
            if c < n_chunks: got.append(c)
        b['need'] = rnd.randint(0, 64)
        if b['part'] >= 64 and b['end'] - b['next'] == 0:
            active.remove(wi)
    assert sorted(got) == list(range(n_chunks)), (len(got), n_chunks)
    return steps


@pytest.mark.parametrize("n_chunks,lg,gl,grab_min,n_waves", [
    (1000, 6, 8, 128, 50), (20480, 6, 8, 128, 300), (123457, 6, 4, 64, 200),
    (777, 0, 8, 128, 20),  # one partition: the progress-slice mode
    (5, 6, 8, 128, 10),  # fewer chunks than partitions
    (100000, 3, 10, 256, 100), (64 * 256 * 3 + 17, 6, 8, 32, 500)])
def test_every_chunk_once(n_chunks, lg, gl, grab_min, n_waves):
    for seed in range(3):
        run(n_chunks, lg, gl, grab_min, n_waves, seed)
