"""A/B of a speculative TwoLayerLoop (diagnostic): each step also queues the
NEXT PDE step (with this step's dt) and its speed before it waits for this
step's U0, so the QG stream never idles through the host's round trip; the
CFL rule then checks the guess (this experiment raises if dt would change —
the bench's dt never does).  Runs bench.main() with the remaining arguments.
usage: python tools/ab_driver_spec.py [--spec] <bench.py args>"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def spec_step(self):
    self.steps += 1
    if not getattr(self, "_spec", False):
        self.dt, changed = self.model.cfl_rule(self.dt, self.U0, self.cfl_fraction)
        self.model.step(self.dt)
        self.model.max_speed_async()
    self.dts.append(self.dt)
    self.t = self.t + self.dt
    active = self.ens is not None and self.t > self.packet_delay
    if active:
        ny = 2 * self.nx
        if not self.have_cur:
            self.model.snapshot(0, which=1, layer=0, ny_period=ny)
        self.model.snapshot(self.group.next_slot(), which=0, layer=0, ny_period=ny)
        self.have_cur = True
        self.group.add(self.dt)
    else:
        self.have_cur = False
    # the guess: the next PDE step with this dt, and its speed
    self.model.step(self.dt)
    self.model.max_speed_async()
    self.U0 = self.model.max_speed_result()  # this step's U0 (the oldest pending)
    dt_next, changed = self.model.cfl_rule(self.dt, self.U0, self.cfl_fraction)
    if changed:
        raise RuntimeError("dt changed: this experiment has no rollback")
    self._spec = True
    return active


if __name__ == "__main__":
    argv = sys.argv[1:]
    spec = "--spec" in argv
    argv = [a for a in argv if a != "--spec"]
    import bench
    bench._imports()
    if spec:
        bench.sw.TwoLayerLoop.step = spec_step
    sys.exit(bench.main(argv))
