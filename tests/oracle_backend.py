"""Test infrastructure: the C oracle behind the controller mirror's context interface.

`ParticleSystemController(backend=oracle_backend(O))` runs the reference controller's host logic (timers,
SplitCell, ProcessPendingSplits, the CellAdhesionManager mirror) with every GPU call replaced by the oracle's
restatement of the same HLSL (oracle/contact_oracle.c: InitParticles, the split edit, the contact step with
adhesion). A GPU run and this replay take identical host decisions exactly when the GPU's particles equal
the oracle's bit for bit, so comparing the two runs frame by frame checks the whole Model R path with bonds
created and moved by division (tests/test_gpu_shipped_bonds.py). Used only by tests.
"""
import numpy as np


class _Stats:
    def __init__(self, capacity, active, steps):
        self.capacity, self.active, self.steps = capacity, active, steps


def oracle_backend(O):
    """A factory (model, dim, capacity, device) -> OracleContext for ParticleSystemController(backend=)."""
    def make(model, dim, capacity, device):
        return OracleContext(O, capacity)
    return make


class OracleContext:
    def __init__(self, O, capacity):
        from sph_test_amd import _abi as A
        self.O, self.A = O, A
        self.capacity = capacity
        self.n = 0
        self.parts = np.zeros(0, O.PARTICLE84)
        self.params = A.SphParams()
        self.conns = None
        self.drag = (-1, (0.0, 0.0, 0.0), 0.0)
        self.steps = 0

    # ------------------------------------------------------------------ params / state
    def get_params(self):
        p = self.A.SphParams()
        for f, _ in p._fields_:
            v = getattr(self.params, f)
            setattr(p, f, v if not hasattr(v, "_length_") else type(v)(*v))
        return p

    def set_params(self, p):
        self.params = p

    def upload_aos84(self, parts):
        self.parts = np.ascontiguousarray(parts).view(self.O.PARTICLE84).copy()
        self.n = len(self.parts)

    def download_aos84(self):
        return self.parts[: self.n].view(self.A.PARTICLE84).copy()

    def get_particles(self, first, count):
        return self.parts[first:first + count].view(self.A.PARTICLE84).copy()

    def set_particles(self, first, parts):
        self.parts[first:first + len(parts)] = np.ascontiguousarray(parts).view(self.O.PARTICLE84)

    def init_particles(self, count, active, genome_modes=0, default_mode=0):
        p = self.params
        self.parts = self.O.init_particles(count, active, p.spawn_radius, p.min_radius, p.max_radius, p.density,
                                           genome_modes, default_mode)
        self.n = count

    def split_particles(self, splits):
        act = self._active()
        need = act + len(splits)
        if need > self.capacity:   # sph_split_particles grows to max(active + count, 2 * capacity)
            self.resize(max(need, 2 * self.capacity))
        out, new_active = self.O.split_particles(self.parts, act, np.ascontiguousarray(splits).view(self.O.SPLIT92))
        self.parts = out[: self.capacity]
        self.n = max(self.n, new_active)
        return new_active

    def resize(self, capacity):
        grown = np.zeros(capacity, self.O.PARTICLE84)
        k = min(capacity, len(self.parts))
        grown[:k] = self.parts[:k]
        self.parts, self.capacity, self.n = grown, capacity, min(self.n, capacity) if capacity < self.n else self.n

    def stats(self):
        return _Stats(self.capacity, self._active(), self.steps)

    def _active(self):
        a = int(self.params.active_particle_count)
        return self.n if a <= 0 or a > self.n else a

    # ------------------------------------------------------------------ step
    def set_adhesion(self, conns):
        self.conns = None if conns is None or len(conns) == 0 else np.ascontiguousarray(conns).view(self.O.ADHESION84).copy()

    def set_drag(self, selected_id, target, strength):
        self.drag = (int(selected_id), tuple(float(t) for t in target), float(strength))

    def step(self, dt, nsteps=1):
        p = self.params
        act = self._active()
        for _ in range(nsteps):
            cp = self.O.contact_params(dt, spawn_radius=p.spawn_radius, global_drag=p.global_drag_multiplier,
                                       torque_factor=p.torque_factor, torque_damping=p.torque_damping,
                                       boundary_friction=p.boundary_friction,
                                       roll_mult=p.rolling_contact_radius_multiplier,
                                       repulsion_strength=p.repulsion_strength, drag_id=self.drag[0],
                                       drag_target=self.drag[1], drag_strength=self.drag[2])
            if self.drag[0] >= act and self.drag[0] < self.n:
                raise NotImplementedError("drag on an inactive particle: not replayed")
            if self.conns is not None:
                if (self.conns["particleA"] >= act).any() or (self.conns["particleB"] >= act).any():
                    raise NotImplementedError("bonds to inactive particles: not replayed")
                out, _, _ = self.O.contact_step_bonds(cp, self.parts[:act], self.conns)
            else:
                out, _ = self.O.contact_step(cp, self.parts[:act])
            self.parts[:act] = out
            self.steps += 1

    # ------------------------------------------------------------------ reads
    def positions(self):
        return np.ascontiguousarray(self.parts["position"][: self.n], dtype=np.float32)

    def rotations(self):
        return np.ascontiguousarray(self.parts["rotation"][: self.n], dtype=np.float32)

    def close(self):
        pass
