"""Legged-locomotion problem builders with the reference's Python API.

Attribution: the phase sequences, cost sets, weights and reference trajectories
below restate Crocoddyl's gait builders (bindings/python/crocoddyl/utils/biped.py
and quadruped.py), Copyright (C) 2018-2020, LAAS-CNRS, University of Edinburgh,
BSD-3-Clause license. They are the workload definition of the C4 / C5 benchmarks
and must reproduce the reference's knot sequences exactly, so the structure and
identifiers follow the original.

Mirrors bindings/python/crocoddyl/utils/biped.py (SimpleBipedGaitProblem, the
Talos walking / jumping problems of benchmark/bipedal_walk_optctrl.py and
bipedal-timings.cpp) and bindings/python/crocoddyl/utils/quadruped.py
(SimpleQuadrupedalGaitProblem, the walking / trotting / pacing / bounding /
jumping gaits of benchmark/quadrupedal_gaits_optctrl.py) on the device-covered
models of crocoddyl_amd.multibody: the same phase sequences, contact models,
costs, weights and reference trajectories, knot by knot.

Differences, each forced by what is absent offline or by a reference defect:
  * Pinocchio is absent: forward kinematics / centre of mass come from
    ``RobotModel.framePlacement`` / ``centerOfMass`` (the same quantities
    pinocchio.updateFramePlacements / centerOfMass return);
  * ``np.asscalar`` (removed from numpy) is ``float``;
  * the quadruped's ``stateBounds`` barrier (quadruped.py:449-454) feeds
    ActivationBounds with the free-flyer's infinite limits, whose midpoint is NaN
    in the reference (quadratic-barrier.hpp:53-57), so the barrier's value there
    depends on Eigen's vectorisation. It is built here only when the robot carries
    finite joint limits, with the free-flyer rows bounded by +-DBL_MAX (the
    vectorised reference's behaviour: those rows never activate);
  * ``x0`` may carry a leading batch axis (B, nx): the gait geometry (feet, CoM)
    comes from x0[0], and the ShootingProblem holds every row as its own element.
"""
import numpy as np

from . import multibody as mb
from .models import IntegratedActionModelEuler


def _problem(x0, running, terminal):
    from .problem import ShootingProblem
    return ShootingProblem(x0, running, terminal)


def _geom_q(x0, nq):
    x0 = np.asarray(x0, float)
    return (x0[0] if x0.ndim == 2 else x0)[:nq]


class SimpleBipedGaitProblem:
    """Defines a simple 3d locomotion problem (utils/biped.py:6-308)."""

    def __init__(self, rmodel, rightFoot, leftFoot):
        self.rmodel = rmodel
        self.state = mb.StateMultibody(self.rmodel)
        self.actuation = mb.ActuationModelFloatingBase(self.state)
        self.rfId = self.rmodel.getFrameId(rightFoot)
        self.lfId = self.rmodel.getFrameId(leftFoot)
        q0 = self.rmodel.referenceConfigurations["half_sitting"]
        self.rmodel.defaultState = np.concatenate([q0, np.zeros(self.rmodel.nv)])
        self.firstStep = True
        self.mu = 0.7
        self.nsurf = np.array([0., 0., 1.])

    def createWalkingModels(self, x0, stepLength, stepHeight, timeStep, stepKnots, supportKnots):
        """The running models of createWalkingProblem (biped.py:25-65)."""
        q0 = _geom_q(x0, self.state.nq)
        rfPos0 = self.rmodel.framePlacement(q0, self.rfId).translation.copy()
        lfPos0 = self.rmodel.framePlacement(q0, self.lfId).translation.copy()
        comRef = (rfPos0 + lfPos0) / 2
        comRef[2] = float(self.rmodel.centerOfMass(q0)[2])
        loco3dModel = []
        doubleSupport = [self.createSwingFootModel(timeStep, [self.rfId, self.lfId]) for k in range(supportKnots)]
        if self.firstStep is True:
            rStep = self.createFootstepModels(comRef, [rfPos0], 0.5 * stepLength, stepHeight, timeStep, stepKnots,
                                              [self.lfId], [self.rfId])
            self.firstStep = False
        else:
            rStep = self.createFootstepModels(comRef, [rfPos0], stepLength, stepHeight, timeStep, stepKnots,
                                              [self.lfId], [self.rfId])
        lStep = self.createFootstepModels(comRef, [lfPos0], stepLength, stepHeight, timeStep, stepKnots, [self.rfId],
                                          [self.lfId])
        loco3dModel += doubleSupport + rStep
        loco3dModel += doubleSupport + lStep
        return loco3dModel

    def createWalkingProblem(self, x0, stepLength, stepHeight, timeStep, stepKnots, supportKnots):
        """Shooting problem for a simple walking gait (biped.py:25-65): double support,
        right step (swing knots + foot switch), double support, left step; the last
        (foot-switch) model is also the terminal one."""
        models = self.createWalkingModels(x0, stepLength, stepHeight, timeStep, stepKnots, supportKnots)
        return _problem(x0, models, models[-1])

    def createJumpingProblem(self, x0, jumpHeight, jumpLength, timeStep, groundKnots, flyingKnots, final=False):
        """biped.py:67-115 (impulse landing)."""
        q0 = _geom_q(x0, self.state.nq)
        rfFootPos0 = self.rmodel.framePlacement(q0, self.rfId).translation.copy()
        lfFootPos0 = self.rmodel.framePlacement(q0, self.lfId).translation.copy()
        jumpLength = np.array(jumpLength, float)
        df = jumpLength[2] - rfFootPos0[2]
        rfFootPos0[2] = 0.
        lfFootPos0[2] = 0.
        comRef = (rfFootPos0 + lfFootPos0) / 2
        comRef[2] = float(self.rmodel.centerOfMass(q0)[2])
        self.rWeight = 1e1
        loco3dModel = []
        takeOff = [self.createSwingFootModel(timeStep, [self.lfId, self.rfId]) for k in range(groundKnots)]
        flyingUpPhase = [
            self.createSwingFootModel(
                timeStep, [],
                np.array([jumpLength[0], jumpLength[1], jumpLength[2] + jumpHeight]) * (k + 1) / flyingKnots + comRef)
            for k in range(flyingKnots)
        ]
        flyingDownPhase = [self.createSwingFootModel(timeStep, []) for k in range(flyingKnots)]
        f0 = jumpLength
        # biped.py:96-99 adds f0 to the frame *ids* (a reference defect); the feet's own
        # positions are used here, as quadruped.py:334-339 does
        footTask = [mb.FramePlacement(self.lfId, mb.SE3(np.eye(3), lfFootPos0 + f0)),
                    mb.FramePlacement(self.rfId, mb.SE3(np.eye(3), rfFootPos0 + f0))]
        landingPhase = [self.createFootSwitchModel([self.lfId, self.rfId], footTask, False)]
        f0[2] = df
        if final is True:
            self.rWeight = 1e4
        landed = [self.createSwingFootModel(timeStep, [self.lfId, self.rfId], comTask=comRef + f0)
                  for k in range(groundKnots)]
        loco3dModel += takeOff + flyingUpPhase + flyingDownPhase + landingPhase + landed
        return _problem(x0, loco3dModel, loco3dModel[-1])

    def createFootstepModels(self, comPos0, feetPos0, stepLength, stepHeight, timeStep, numKnots, supportFootIds,
                             swingFootIds):
        """Action models for a footstep phase (biped.py:117-168); comPos0 and
        feetPos0 are advanced in place, as in the reference."""
        numLegs = len(supportFootIds) + len(swingFootIds)
        comPercentage = float(len(swingFootIds)) / numLegs
        footSwingModel = []
        for k in range(numKnots):
            swingFootTask = []
            for i, p in zip(swingFootIds, feetPos0):
                phKnots = numKnots / 2
                if k < phKnots:
                    dp = np.array([stepLength * (k + 1) / numKnots, 0., stepHeight * k / phKnots])
                elif k == phKnots:
                    dp = np.array([stepLength * (k + 1) / numKnots, 0., stepHeight])
                else:
                    dp = np.array(
                        [stepLength * (k + 1) / numKnots, 0., stepHeight * (1 - float(k - phKnots) / phKnots)])
                tref = p + dp
                swingFootTask += [mb.FramePlacement(i, mb.SE3(np.eye(3), tref))]
            comTask = np.array([stepLength * (k + 1) / numKnots, 0., 0.]) * comPercentage + comPos0
            footSwingModel += [
                self.createSwingFootModel(timeStep, supportFootIds, comTask=comTask, swingFootTask=swingFootTask)
            ]
        footSwitchModel = self.createFootSwitchModel(supportFootIds, swingFootTask)
        comPos0 += [stepLength * comPercentage, 0., 0.]
        for p in feetPos0:
            p += [stepLength, 0., 0.]
        return footSwingModel + [footSwitchModel]

    def _stateReg(self, weights, nu):
        return mb.CostModelState(self.state, mb.ActivationModelWeightedQuad(weights**2), self.rmodel.defaultState, nu)

    def _cones(self, costModel, supportFootIds):
        for i in supportFootIds:
            cone = mb.FrictionCone(self.nsurf, self.mu, 4, False)
            frictionCone = mb.CostModelContactFrictionCone(
                self.state, mb.ActivationModelQuadraticBarrier(mb.ActivationBounds(cone.lb, cone.ub)),
                mb.FrameFrictionCone(i, cone), self.actuation.nu)
            costModel.addCost(self.rmodel.frames[i][0] + "_frictionCone", frictionCone, 1e1)

    def _contacts6d(self, supportFootIds):
        contactModel = mb.ContactModelMultiple(self.state, self.actuation.nu)
        for i in supportFootIds:
            Mref = mb.FramePlacement(i, mb.SE3.Identity())
            supportContactModel = mb.ContactModel6D(self.state, Mref, self.actuation.nu, np.array([0., 0.]))
            contactModel.addContact(self.rmodel.frames[i][0] + "_contact", supportContactModel)
        return contactModel

    def createSwingFootModel(self, timeStep, supportFootIds, comTask=None, swingFootTask=None):
        """Action model for a swing foot phase (biped.py:170-216): 6D contacts on the
        support feet, CoM (1e6), friction cones (1e1), swing-foot placements (1e6),
        state (1e1) and control (1e-1) regularisation; Euler(timeStep)."""
        contactModel = self._contacts6d(supportFootIds)
        costModel = mb.CostModelSum(self.state, self.actuation.nu)
        if isinstance(comTask, np.ndarray):
            comTrack = mb.CostModelCoMPosition(self.state, comTask, self.actuation.nu)
            costModel.addCost("comTrack", comTrack, 1e6)
        self._cones(costModel, supportFootIds)
        if swingFootTask is not None:
            for i in swingFootTask:
                footTrack = mb.CostModelFramePlacement(self.state, i, self.actuation.nu)
                costModel.addCost(self.rmodel.frames[i.id][0] + "_footTrack", footTrack, 1e6)
        stateWeights = np.array([0] * 3 + [500.] * 3 + [0.01] * (self.state.nv - 6) + [10] * self.state.nv)
        costModel.addCost("stateReg", self._stateReg(stateWeights, self.actuation.nu), 1e1)
        costModel.addCost("ctrlReg", mb.CostModelControl(self.state, self.actuation.nu), 1e-1)
        dmodel = mb.DifferentialActionModelContactFwdDynamics(self.state, self.actuation, contactModel, costModel,
                                                              0., True)
        return IntegratedActionModelEuler(dmodel, timeStep)

    def createFootSwitchModel(self, supportFootIds, swingFootTask, pseudoImpulse=True):
        """Foot switch (biped.py:218-229): pseudo-impulse by default."""
        if pseudoImpulse:
            return self.createPseudoImpulseModel(supportFootIds, swingFootTask)
        return self.createImpulseModel(supportFootIds, swingFootTask)

    def createPseudoImpulseModel(self, supportFootIds, swingFootTask):
        """biped.py:231-276: high penalties on the swing feet's placement (1e8) and
        velocity (1e6), Euler with dt = 0."""
        contactModel = self._contacts6d(supportFootIds)
        costModel = mb.CostModelSum(self.state, self.actuation.nu)
        self._cones(costModel, supportFootIds)
        if swingFootTask is not None:
            for i in swingFootTask:
                footTrack = mb.CostModelFramePlacement(self.state, i, self.actuation.nu)
                costModel.addCost(self.rmodel.frames[i.id][0] + "_footTrack", footTrack, 1e8)
                footVel = mb.FrameMotion(i.id, mb.Motion.Zero())
                impulseFootVelCost = mb.CostModelFrameVelocity(self.state, footVel, self.actuation.nu)
                costModel.addCost(self.rmodel.frames[i.id][0] + "_impulseVel", impulseFootVelCost, 1e6)
        stateWeights = np.array([0] * 3 + [500.] * 3 + [0.01] * (self.state.nv - 6) + [10] * self.state.nv)
        costModel.addCost("stateReg", self._stateReg(stateWeights, self.actuation.nu), 1e1)
        costModel.addCost("ctrlReg", mb.CostModelControl(self.state, self.actuation.nu), 1e-3)
        dmodel = mb.DifferentialActionModelContactFwdDynamics(self.state, self.actuation, contactModel, costModel,
                                                              0., True)
        return IntegratedActionModelEuler(dmodel, 0.)

    def createImpulseModel(self, supportFootIds, swingFootTask):
        """biped.py:278-307: ImpulseModel6D on the support feet, swing-foot
        translations (1e8), state regularisation (1e1)."""
        impulseModel = mb.ImpulseModelMultiple(self.state)
        for i in supportFootIds:
            impulseModel.addImpulse(self.rmodel.frames[i][0] + "_impulse", mb.ImpulseModel6D(self.state, i))
        costModel = mb.CostModelSum(self.state, 0)
        if swingFootTask is not None:
            for i in swingFootTask:
                xref = mb.FrameTranslation(i.id, i.oMf.translation)
                footTrack = mb.CostModelFrameTranslation(self.state, xref, 0)
                costModel.addCost(self.rmodel.frames[i.id][0] + "_footTrack", footTrack, 1e8)
        stateWeights = np.array([1.] * 6 + [0.1] * (self.rmodel.nv - 6) + [10] * self.rmodel.nv)
        costModel.addCost("stateReg", self._stateReg(stateWeights, 0), 1e1)
        return mb.ActionModelImpulseFwdDynamics(self.state, impulseModel, costModel)


class SimpleQuadrupedalGaitProblem:
    """utils/quadruped.py:6-553."""

    def __init__(self, rmodel, lfFoot, rfFoot, lhFoot, rhFoot):
        self.rmodel = rmodel
        self.state = mb.StateMultibody(self.rmodel)
        self.actuation = mb.ActuationModelFloatingBase(self.state)
        self.lfFootId = self.rmodel.getFrameId(lfFoot)
        self.rfFootId = self.rmodel.getFrameId(rfFoot)
        self.lhFootId = self.rmodel.getFrameId(lhFoot)
        self.rhFootId = self.rmodel.getFrameId(rhFoot)
        q0 = self.rmodel.referenceConfigurations["standing"]
        self.rmodel.defaultState = np.concatenate([q0, np.zeros(self.rmodel.nv)])
        self.firstStep = True
        self.mu = 0.7
        self.nsurf = np.array([0., 0., 1.])

    @property
    def _all(self):
        return [self.lfFootId, self.rfFootId, self.lhFootId, self.rhFootId]

    def _feet(self, x0):
        q0 = _geom_q(x0, self.state.nq)
        pos = [self.rmodel.framePlacement(q0, f).translation.copy()
               for f in (self.rfFootId, self.rhFootId, self.lfFootId, self.lhFootId)]
        comRef = sum(pos) / 4
        comRef[2] = float(self.rmodel.centerOfMass(q0)[2])
        return pos, comRef

    def createCoMProblem(self, x0, comGoTo, timeStep, numKnots):
        """quadruped.py:25-72."""
        com0 = self.rmodel.centerOfMass(_geom_q(x0, self.state.nq))
        fwd = [self.createSwingFootModel(timeStep, self._all) for k in range(numKnots)]
        fwdTerm = self.createSwingFootModel(timeStep, self._all, com0 + np.array([comGoTo, 0., 0.]))
        fwdTerm.differential.costs.costs['comTrack'].weight = 1e6
        bwd = [self.createSwingFootModel(timeStep, self._all) for k in range(numKnots)]
        bwdTerm = self.createSwingFootModel(timeStep, self._all, com0 + np.array([-comGoTo, 0., 0.]))
        bwdTerm.differential.costs.costs['comTrack'].weight = 1e6
        comModels = fwd + [fwdTerm] + bwd + [bwdTerm]
        return _problem(x0, comModels, comModels[-1])

    def createWalkingModels(self, x0, stepLength, stepHeight, timeStep, stepKnots, supportKnots):
        """quadruped.py:111-160 (running models)."""
        (rfFootPos0, rhFootPos0, lfFootPos0, lhFootPos0), comRef = self._feet(x0)
        doubleSupport = [self.createSwingFootModel(timeStep, self._all) for k in range(supportKnots)]
        sl = 0.5 * stepLength if self.firstStep is True else stepLength
        rhStep = self.createFootstepModels(comRef, [rhFootPos0], sl, stepHeight, timeStep, stepKnots,
                                           [self.lfFootId, self.rfFootId, self.lhFootId], [self.rhFootId])
        rfStep = self.createFootstepModels(comRef, [rfFootPos0], sl, stepHeight, timeStep, stepKnots,
                                           [self.lfFootId, self.lhFootId, self.rhFootId], [self.rfFootId])
        self.firstStep = False
        lhStep = self.createFootstepModels(comRef, [lhFootPos0], stepLength, stepHeight, timeStep, stepKnots,
                                           [self.lfFootId, self.rfFootId, self.rhFootId], [self.lhFootId])
        lfStep = self.createFootstepModels(comRef, [lfFootPos0], stepLength, stepHeight, timeStep, stepKnots,
                                           [self.rfFootId, self.lhFootId, self.rhFootId], [self.lfFootId])
        return doubleSupport + rhStep + rfStep + doubleSupport + lhStep + lfStep

    def createWalkingProblem(self, x0, stepLength, stepHeight, timeStep, stepKnots, supportKnots):
        models = self.createWalkingModels(x0, stepLength, stepHeight, timeStep, stepKnots, supportKnots)
        return _problem(x0, models, models[-1])

    def createTrottingModels(self, x0, stepLength, stepHeight, timeStep, stepKnots, supportKnots):
        """quadruped.py:162-208 (running models): diagonal pairs RF+LH, then LF+RH."""
        (rfFootPos0, rhFootPos0, lfFootPos0, lhFootPos0), comRef = self._feet(x0)
        doubleSupport = [self.createSwingFootModel(timeStep, self._all) for k in range(supportKnots)]
        sl = 0.5 * stepLength if self.firstStep is True else stepLength
        rflhStep = self.createFootstepModels(comRef, [rfFootPos0, lhFootPos0], sl, stepHeight, timeStep, stepKnots,
                                             [self.lfFootId, self.rhFootId], [self.rfFootId, self.lhFootId])
        self.firstStep = False
        lfrhStep = self.createFootstepModels(comRef, [lfFootPos0, rhFootPos0], stepLength, stepHeight, timeStep,
                                             stepKnots, [self.rfFootId, self.lhFootId], [self.lfFootId, self.rhFootId])
        return doubleSupport + rflhStep + doubleSupport + lfrhStep

    def createTrottingProblem(self, x0, stepLength, stepHeight, timeStep, stepKnots, supportKnots):
        models = self.createTrottingModels(x0, stepLength, stepHeight, timeStep, stepKnots, supportKnots)
        return _problem(x0, models, models[-1])

    def createPacingProblem(self, x0, stepLength, stepHeight, timeStep, stepKnots, supportKnots):
        """quadruped.py:210-257: lateral pairs."""
        (rfFootPos0, rhFootPos0, lfFootPos0, lhFootPos0), comRef = self._feet(x0)
        doubleSupport = [self.createSwingFootModel(timeStep, self._all) for k in range(supportKnots)]
        sl = 0.5 * stepLength if self.firstStep is True else stepLength
        rightSteps = self.createFootstepModels(comRef, [rfFootPos0, rhFootPos0], sl, stepHeight, timeStep, stepKnots,
                                               [self.lfFootId, self.lhFootId], [self.rfFootId, self.rhFootId])
        self.firstStep = False
        leftSteps = self.createFootstepModels(comRef, [lfFootPos0, lhFootPos0], stepLength, stepHeight, timeStep,
                                              stepKnots, [self.rfFootId, self.rhFootId], [self.lfFootId, self.lhFootId])
        models = doubleSupport + rightSteps + doubleSupport + leftSteps
        return _problem(x0, models, models[-1])

    def createBoundingProblem(self, x0, stepLength, stepHeight, timeStep, stepKnots, supportKnots):
        """quadruped.py:259-298: front / hind pairs."""
        (rfFootPos0, rhFootPos0, lfFootPos0, lhFootPos0), comRef = self._feet(x0)
        doubleSupport = [self.createSwingFootModel(timeStep, self._all) for k in range(supportKnots)]
        hindSteps = self.createFootstepModels(comRef, [lfFootPos0, rfFootPos0], stepLength, stepHeight, timeStep,
                                              stepKnots, [self.lhFootId, self.rhFootId], [self.lfFootId, self.rfFootId])
        frontSteps = self.createFootstepModels(comRef, [lhFootPos0, rhFootPos0], stepLength, stepHeight, timeStep,
                                               stepKnots, [self.lfFootId, self.rfFootId],
                                               [self.lhFootId, self.rhFootId])
        models = doubleSupport + hindSteps + doubleSupport + frontSteps
        return _problem(x0, models, models[-1])

    def createJumpingProblem(self, x0, jumpHeight, jumpLength, timeStep, groundKnots, flyingKnots):
        """quadruped.py:300-355."""
        (rfFootPos0, rhFootPos0, lfFootPos0, lhFootPos0), _ = self._feet(x0)
        q0 = _geom_q(x0, self.state.nq)
        jumpLength = np.array(jumpLength, float)
        df = jumpLength[2] - rfFootPos0[2]
        for p in (rfFootPos0, rhFootPos0, lfFootPos0, lhFootPos0):
            p[2] = 0.
        comRef = (rfFootPos0 + rhFootPos0 + lfFootPos0 + lhFootPos0) / 4
        comRef[2] = float(self.rmodel.centerOfMass(q0)[2])
        takeOff = [self.createSwingFootModel(timeStep, self._all) for k in range(groundKnots)]
        flyingUpPhase = [
            self.createSwingFootModel(
                timeStep, [],
                np.array([jumpLength[0], jumpLength[1], jumpLength[2] + jumpHeight]) * (k + 1) / flyingKnots + comRef)
            for k in range(flyingKnots)
        ]
        flyingDownPhase = [self.createSwingFootModel(timeStep, []) for k in range(flyingKnots)]
        f0 = jumpLength
        footTask = [mb.FramePlacement(self.lfFootId, mb.SE3(np.eye(3), lfFootPos0 + f0)),
                    mb.FramePlacement(self.rfFootId, mb.SE3(np.eye(3), rfFootPos0 + f0)),
                    mb.FramePlacement(self.lhFootId, mb.SE3(np.eye(3), lhFootPos0 + f0)),
                    mb.FramePlacement(self.rhFootId, mb.SE3(np.eye(3), rhFootPos0 + f0))]
        landingPhase = [self.createFootSwitchModel(self._all, footTask, False)]
        f0[2] = df
        landed = [self.createSwingFootModel(timeStep, self._all, comTask=comRef + f0) for k in range(groundKnots)]
        models = takeOff + flyingUpPhase + flyingDownPhase + landingPhase + landed
        return _problem(x0, models, models[-1])

    def createFootstepModels(self, comPos0, feetPos0, stepLength, stepHeight, timeStep, numKnots, supportFootIds,
                             swingFootIds):
        """quadruped.py:357-405 (comPos0 / feetPos0 advanced in place)."""
        numLegs = len(supportFootIds) + len(swingFootIds)
        comPercentage = float(len(swingFootIds)) / numLegs
        footSwingModel = []
        for k in range(numKnots):
            swingFootTask = []
            for i, p in zip(swingFootIds, feetPos0):
                phKnots = numKnots / 2
                if k < phKnots:
                    dp = np.array([stepLength * (k + 1) / numKnots, 0., stepHeight * k / phKnots])
                elif k == phKnots:
                    dp = np.array([stepLength * (k + 1) / numKnots, 0., stepHeight])
                else:
                    dp = np.array(
                        [stepLength * (k + 1) / numKnots, 0., stepHeight * (1 - float(k - phKnots) / phKnots)])
                tref = p + dp
                swingFootTask += [mb.FramePlacement(i, mb.SE3(np.eye(3), tref))]
            comTask = np.array([stepLength * (k + 1) / numKnots, 0., 0.]) * comPercentage + comPos0
            footSwingModel += [
                self.createSwingFootModel(timeStep, supportFootIds, comTask=comTask, swingFootTask=swingFootTask)
            ]
        footSwitchModel = self.createFootSwitchModel(supportFootIds, swingFootTask)
        comPos0 += [stepLength * comPercentage, 0., 0.]
        for p in feetPos0:
            p += [stepLength, 0., 0.]
        return footSwingModel + [footSwitchModel]

    def _contacts3d(self, supportFootIds):
        contactModel = mb.ContactModelMultiple(self.state, self.actuation.nu)
        for i in supportFootIds:
            xref = mb.FrameTranslation(i, np.array([0., 0., 0.]))
            supportContactModel = mb.ContactModel3D(self.state, xref, self.actuation.nu, np.array([0., 50.]))
            contactModel.addContact(self.rmodel.frames[i][0] + "_contact", supportContactModel)
        return contactModel

    def _cones(self, costModel, supportFootIds):
        for i in supportFootIds:
            cone = mb.FrictionCone(self.nsurf, self.mu, 4, False)
            frictionCone = mb.CostModelContactFrictionCone(
                self.state, mb.ActivationModelQuadraticBarrier(mb.ActivationBounds(cone.lb, cone.ub)),
                mb.FrameFrictionCone(i, cone), self.actuation.nu)
            costModel.addCost(self.rmodel.frames[i][0] + "_frictionCone", frictionCone, 1e1)

    def _stateReg(self, weights, nu):
        return mb.CostModelState(self.state, mb.ActivationModelWeightedQuad(weights**2), self.rmodel.defaultState, nu)

    def createSwingFootModel(self, timeStep, supportFootIds, comTask=None, swingFootTask=None):
        """quadruped.py:407-461: 3D contacts (gains [0, 50]) on the support feet,
        CoM (1e6), friction cones (1e1), swing-foot translations (1e6), state (1e1)
        and control (1e-1) regularisation, state bounds (1e3, see the module note)."""
        contactModel = self._contacts3d(supportFootIds)
        costModel = mb.CostModelSum(self.state, self.actuation.nu)
        if isinstance(comTask, np.ndarray):
            comTrack = mb.CostModelCoMPosition(self.state, comTask, self.actuation.nu)
            costModel.addCost("comTrack", comTrack, 1e6)
        self._cones(costModel, supportFootIds)
        if swingFootTask is not None:
            for i in swingFootTask:
                xref = mb.FrameTranslation(i.id, i.placement.translation)
                footTrack = mb.CostModelFrameTranslation(self.state, xref, self.actuation.nu)
                costModel.addCost(self.rmodel.frames[i.id][0] + "_footTrack", footTrack, 1e6)
        nv = self.rmodel.nv
        stateWeights = np.array([0.] * 3 + [500.] * 3 + [0.01] * (nv - 6) + [10.] * 6 + [1.] * (nv - 6))
        costModel.addCost("stateReg", self._stateReg(stateWeights, self.actuation.nu), 1e1)
        costModel.addCost("ctrlReg", mb.CostModelControl(self.state, self.actuation.nu), 1e-1)
        if np.all(np.isfinite(self.state.lb[7:self.state.nq])):  # finite joint position limits (module note)
            lb = np.concatenate([self.state.lb[1:nv + 1], self.state.lb[-nv:]])
            ub = np.concatenate([self.state.ub[1:nv + 1], self.state.ub[-nv:]])
            lb, ub = np.nan_to_num(lb, neginf=-mb.DBL_MAX), np.nan_to_num(ub, posinf=mb.DBL_MAX)
            stateBounds = mb.CostModelState(
                self.state, mb.ActivationModelQuadraticBarrier(mb.ActivationBounds(lb, ub)),
                0 * self.rmodel.defaultState, self.actuation.nu)
            costModel.addCost("stateBounds", stateBounds, 1e3)
        dmodel = mb.DifferentialActionModelContactFwdDynamics(self.state, self.actuation, contactModel, costModel,
                                                              0., True)
        return IntegratedActionModelEuler(dmodel, timeStep)

    def createFootSwitchModel(self, supportFootIds, swingFootTask, pseudoImpulse=False):
        """quadruped.py:463-474: an impulse model by default."""
        if pseudoImpulse:
            return self.createPseudoImpulseModel(supportFootIds, swingFootTask)
        return self.createImpulseModel(supportFootIds, swingFootTask)

    def createPseudoImpulseModel(self, supportFootIds, swingFootTask):
        """quadruped.py:476-520."""
        contactModel = self._contacts3d(supportFootIds)
        costModel = mb.CostModelSum(self.state, self.actuation.nu)
        self._cones(costModel, supportFootIds)
        if swingFootTask is not None:
            for i in swingFootTask:
                xref = mb.FrameTranslation(i.frame, i.oMf.translation)
                vref = mb.FrameMotion(i.frame, mb.Motion.Zero())
                footTrack = mb.CostModelFrameTranslation(self.state, xref, self.actuation.nu)
                impulseFootVelCost = mb.CostModelFrameVelocity(self.state, vref, self.actuation.nu)
                costModel.addCost(self.rmodel.frames[i.frame][0] + "_footTrack", footTrack, 1e7)
                costModel.addCost(self.rmodel.frames[i.frame][0] + "_impulseVel", impulseFootVelCost, 1e6)
        nv = self.rmodel.nv
        stateWeights = np.array([0.] * 3 + [500.] * 3 + [0.01] * (nv - 6) + [10.] * nv)
        costModel.addCost("stateReg", self._stateReg(stateWeights, self.actuation.nu), 1e1)
        costModel.addCost("ctrlReg", mb.CostModelControl(self.state, self.actuation.nu), 1e-3)
        dmodel = mb.DifferentialActionModelContactFwdDynamics(self.state, self.actuation, contactModel, costModel,
                                                              0., True)
        return IntegratedActionModelEuler(dmodel, 0.)

    def createImpulseModel(self, supportFootIds, swingFootTask, JMinvJt_damping=1e-12, r_coeff=0.0):
        """quadruped.py:522-553: ImpulseModel3D on the support feet."""
        impulseModel = mb.ImpulseModelMultiple(self.state)
        for i in supportFootIds:
            impulseModel.addImpulse(self.rmodel.frames[i][0] + "_impulse", mb.ImpulseModel3D(self.state, i))
        costModel = mb.CostModelSum(self.state, 0)
        if swingFootTask is not None:
            for i in swingFootTask:
                xref = mb.FrameTranslation(i.id, i.oMf.translation)
                footTrack = mb.CostModelFrameTranslation(self.state, xref, 0)
                costModel.addCost(self.rmodel.frames[i.id][0] + "_footTrack", footTrack, 1e7)
        nv = self.rmodel.nv
        stateWeights = np.array([1.] * 6 + [10.] * (nv - 6) + [10.] * nv)
        costModel.addCost("stateReg", self._stateReg(stateWeights, 0), 1e1)
        model = mb.ActionModelImpulseFwdDynamics(self.state, impulseModel, costModel)
        model.JMinvJt_damping = JMinvJt_damping
        model.r_coeff = r_coeff
        return model
