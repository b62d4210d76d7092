"""BoxQP / BoxQPSolution with the reference's Python API, solved on the GPU.

Reference: include/crocoddyl/core/solvers/box-qp.hpp:29-206,
src/core/solvers/box-qp.cpp:14-252, bindings/python/crocoddyl/core/solvers/box-qp.cpp.
The projected-Newton iterations run in libfddp_hip (one wave per QP,
crocoddyl_amd/csrc/box_qp.hpp) through fddp_boxqp_solve; a leading batch
axis on H, q, lb, ub, xinit solves B independent QPs in one launch.
"""
import ctypes as C
import warnings

import numpy as np

from . import _abi
from ._lib import FDDPError, check, lib


class BoxQPSolution:
    """BoxQPSolution (box-qp.hpp:29-53): Hff_inv (nf x nf), x, free_idx, clamped_idx."""

    def __init__(self, Hff_inv=None, x=None, free_idx=(), clamped_idx=()):
        self.Hff_inv = np.zeros((0, 0)) if Hff_inv is None else np.asarray(Hff_inv, float)
        self.x = np.zeros(0) if x is None else np.asarray(x, float)
        self.free_idx = list(free_idx)
        self.clamped_idx = list(clamped_idx)


class BoxQP:
    """Projected-Newton QP with bound constraints:
    x = argmin 0.5 x'Hx + q'x  s.t.  lb <= x <= ub   (box-qp.cpp:14-46 defaults)."""

    def __init__(self, nx, maxiter=100, th_acceptstep=0.1, th_grad=1e-9, reg=1e-9, device=0):
        self._p = _abi.BoxQPParams()
        lib().fddp_boxqp_default_params(C.byref(self._p))
        self.nx = int(nx)
        self.maxiter = int(maxiter)
        self._p.th_acceptstep = float(th_acceptstep)
        # the constructor only warns (box-qp.cpp:28-36)
        if th_grad < 0.0:
            warnings.warn("th_grad value has to be positive.")
        if reg < 0.0:
            warnings.warn("reg value has to be positive.")
        self._p.th_grad = float(th_grad)
        self._p.reg = float(reg)
        self.device = int(device)
        self.solution = BoxQPSolution()

    # -- properties with the reference setter validation (box-qp.cpp:199-249) --
    @property
    def maxiter(self):
        return self._p.maxiter

    @maxiter.setter
    def maxiter(self, v):
        self._p.maxiter = int(v)

    @property
    def th_acceptStep(self):
        return self._p.th_acceptstep

    @th_acceptStep.setter
    def th_acceptStep(self, v):
        # box-qp.cpp:203-208 tests `0 >= v && v >= 0.5`, which never holds: no error
        self._p.th_acceptstep = float(v)

    @property
    def th_grad(self):
        return self._p.th_grad

    @th_grad.setter
    def th_grad(self, v):
        if v < 0.0:
            raise FDDPError("Invalid argument: th_grad value has to be positive.")
        self._p.th_grad = float(v)

    @property
    def reg(self):
        return self._p.reg

    @reg.setter
    def reg(self, v):
        if v < 0.0:
            raise FDDPError("Invalid argument: reg value has to be positive.")
        self._p.reg = float(v)

    @property
    def alphas(self):
        return [self._p.alphas[i] for i in range(self._p.n_alphas)]

    @alphas.setter
    def alphas(self, a):
        a = [float(x) for x in a]
        if not a or len(a) > 16:
            raise FDDPError("Invalid argument: between 1 and 16 alphas")
        if a[0] != 1.0:
            warnings.warn("alpha[0] should be 1")
        for i in range(1, len(a)):
            if a[i] <= 0.0:
                raise FDDPError("Invalid argument: alpha values has to be positive.")
            if a[i] >= a[i - 1]:
                raise FDDPError("Invalid argument: alpha values are monotonously decreasing.")
        self._p.n_alphas = len(a)
        for i in range(16):
            self._p.alphas[i] = a[i] if i < len(a) else 0.0

    # -- solve -------------------------------------------------------------------
    def solve(self, H, q, lb, ub, xinit):
        """BoxQP::solve (box-qp.cpp:51-182). With a leading batch axis,
        returns a list of BoxQPSolution (one per problem)."""
        n = self.nx
        H = np.asarray(H, float)
        batched = H.ndim == 3
        B = H.shape[0] if batched else 1
        names = ("q", "lb", "ub", "xinit")
        if H.shape[-2:] != (n, n):
            raise FDDPError(f"Invalid argument: H has wrong dimension (it should be {n},{n})")
        vecs = []
        for name, v in zip(names, (q, lb, ub, xinit)):
            v = np.asarray(v, float)
            if v.shape[-1:] != (n,):
                raise FDDPError(f"Invalid argument: {name} has wrong dimension (it should be {n})")
            vecs.append(np.ascontiguousarray(np.broadcast_to(v, (B, n))))
        Hc = np.ascontiguousarray(np.broadcast_to(H, (B, n, n)).transpose(0, 2, 1))  # column-major blocks
        x = np.zeros((B, n))
        fm = np.zeros(B, dtype=np.uint64)
        im = np.zeros(B, dtype=np.uint64)
        Hi = np.zeros((B, n, n))
        st = np.zeros(B, dtype=np.int32)
        check(lib().fddp_boxqp_solve(self.device, B, n, _abi.dptr(Hc), *[_abi.dptr(v) for v in vecs],
                                     C.byref(self._p), _abi.dptr(x), fm.ctypes.data_as(_abi.U64),
                                     im.ctypes.data_as(_abi.U64), _abi.dptr(Hi), st.ctypes.data_as(_abi.I32)))
        sols = []
        for b in range(B):
            if st[b]:
                if not batched:
                    raise FDDPError("backward_error")
                sols.append(None)
                continue
            free = [i for i in range(n) if (int(fm[b]) >> i) & 1]
            clamped = [i for i in range(n) if not (int(fm[b]) >> i) & 1]
            inv = [i for i in range(n) if (int(im[b]) >> i) & 1]
            Hff = Hi[b].T[np.ix_(inv, inv)]  # column-major block -> (nx, nx), compact on the inverse's free set
            sols.append(BoxQPSolution(Hff, x[b], free, clamped))
        if batched:
            return sols
        self.solution = sols[0]
        return sols[0]
