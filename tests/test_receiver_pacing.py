"""ReceiverLoop's host-side ordering in the PDE-owner form (qg.py), on CPU with
stub link / context / events — no GPU.

With a device link the receivers order the link buffers on the host alone
(OwnerLink.snapshot fenced): step m's broadcast lands in buffer m % nbuf,
step m's snapshot reads it (and, on a first active step, step m + 1's
grid_U(prev_qk) reads it again), and receive m + nbuf refills it.  The loop
waits on the host for the broadcast before queueing a snapshot, and refills a
buffer only after it has synchronised a pacing event recorded after the
packet work of every step that read it.  Here the "device" never finishes
anything on its own: a queued read completes only when the host synchronises
an event recorded after it, so any refill that could race a read is caught."""
import types

import pytest

import swraytracing_amd.qg as qg


class Device:
    """Queued work in stream order; nothing completes until an event behind it
    is synchronised."""

    def __init__(self):
        self.queue = []  # ("read", buf, step) | ("mark", event)
        self.step = 0

    def complete_through(self, ev):
        i = self.queue.index(("mark", ev))
        del self.queue[:i + 1]

    def pending_reads(self, buf):
        return [q for q in self.queue if q[0] == "read" and q[1] == buf]


class StubEvent:
    def __init__(self, dev):
        self.dev = dev

    def record(self, stream):
        self.dev.queue.append(("mark", self))

    def synchronize(self):
        if ("mark", self) in self.dev.queue:
            self.dev.complete_through(self)


class StubLink:
    def __init__(self, dev, nbuf, dts):
        self.dev, self.nbuf, self.dts = dev, nbuf, list(dts)
        self.device = True
        self.cur = 0
        self.landed = {0: True}  # buffer -> its broadcast has completed (host view)
        self.received = 0

    def receive(self, wait=False):
        b = (self.cur + 1) % self.nbuf
        # the refill: nothing queued may still read this buffer
        assert not self.dev.pending_reads(b), (b, self.dev.pending_reads(b))
        self.cur = b
        self.landed[b] = bool(wait)  # a fenced snapshot needs the host to have seen it land
        dt = self.dts[self.received]
        self.received += 1
        return dt

    def snapshot(self, ctx, slot, which, L, K_d2, shear, k_scale, ny_period, fenced=False):
        b = self.cur if which == 0 else (self.cur - 1) % self.nbuf
        assert fenced and self.landed.get(b, False), (b, fenced)
        self.dev.queue.append(("read", b, self.dev.step))


class StubCtx:
    def __init__(self, dev):
        self.dev = dev

    def stream(self):
        return 0

    def swap_slots(self, a, b):
        pass


def _ensemble(dev):
    ctx = StubCtx(dev)
    return types.SimpleNamespace(
        ctx=ctx, n=100, L=20.0, K_d2=3.0, shear=0.5, k_scale=0.3, ny_period=128,
        advance_intervals=lambda dts, nsub: dev.queue.append(("packets", dev.step)))


@pytest.fixture
def stub_torch(monkeypatch):
    import torch
    dev = Device()
    monkeypatch.setattr(torch.cuda, "ExternalStream", lambda s: ("stream", s))
    monkeypatch.setattr(torch.cuda, "Event", lambda *a, **k: StubEvent(dev))
    return dev


@pytest.mark.parametrize("nbuf", [4, 5, 6, 8])
@pytest.mark.parametrize("delay_steps", [0, 3])
def test_receiver_never_refills_a_buffer_a_queued_snapshot_reads(stub_torch, nbuf, delay_steps):
    """Every nbuf >= 4 (the loop's own look-ahead, ahead = nbuf - 3 >= 1) and a
    packet delay (the first active step reads the previous buffer too): every
    refill happens after the host synchronised a pacing event behind every
    read of that buffer, and every snapshot reads a buffer whose broadcast the
    host saw land."""
    dev = stub_torch
    dt = 0.1
    steps = 40
    link = StubLink(dev, nbuf, [dt] * (steps + 1))
    loop = qg.ReceiverLoop(link, _ensemble(dev), dt, packet_delay=(delay_steps + 0.5) * dt, nsub=2)
    assert loop._fenced and loop.ahead == nbuf - loop.mark_every - 1
    active = 0
    for s in range(1, steps + 1):
        dev.step = s
        active += bool(loop.step())
    assert active == steps - delay_steps
    reads = [q for q in dev.queue if q[0] == "read"]
    assert len(reads) <= 2 * nbuf  # the host stays within its look-ahead


@pytest.mark.parametrize("nbuf,ahead", [(3, 2), (5, 3), (3, None)])
def test_receiver_unfenced_when_the_buffers_are_too_few(stub_torch, nbuf, ahead):
    """ahead + mark_every + 1 > nbuf, or no look-ahead at all (3 buffers:
    ahead 0, no pacing): the loop does not claim the host order (its
    snapshots are then ordered by events on the link's stream)."""
    dev = stub_torch
    link = StubLink(dev, nbuf, [0.1] * 4)
    loop = qg.ReceiverLoop(link, _ensemble(dev), 0.1, ahead=ahead)
    assert not loop._fenced
