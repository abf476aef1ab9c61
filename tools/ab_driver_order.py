"""A/B of TwoLayerLoop's queue order (diagnostic): with --old-order the
step queues the speed pass (Jacobian + CFL max + U0 copy) before the grid_U
snapshot, as round 3 did before the reorder, so the packet launch waited
behind the speed pass.  Runs bench.main() with the remaining arguments.
usage: python tools/ab_driver_order.py [--old-order] <bench.py args>"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def old_step(self):
    self.steps += 1
    self.dt, changed = self.model.cfl_rule(self.dt, self.U0, self.cfl_fraction)
    self.dts.append(self.dt)
    self.model.step(self.dt)
    self.t = self.t + self.dt
    self.model.max_speed_async()
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
    self.U0 = self.model.max_speed_result()
    return active


if __name__ == "__main__":
    argv = sys.argv[1:]
    old = "--old-order" in argv
    argv = [a for a in argv if a != "--old-order"]
    import bench
    bench._imports()
    if old:
        bench.sw.TwoLayerLoop.step = old_step
    sys.exit(bench.main(argv))
