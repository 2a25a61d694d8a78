"""The reference's shipped scenario as data, for tests that run where /root/reference is absent
(the GPU box). tests/test_lifecycle_cpu.py checks both against the reference's own files:
`Assets/Scenes/Particle Simulation.unity:151-163` (ParticleSystemController inspector values) and
`Assets/Scripts/Genome System/NewCellGenome.asset:15-38` (one mode)."""

SCENE_CONTROLLER = {
    "particleCount": 4, "minRadius": 2, "maxRadius": 2, "spawnRadius": 15, "globalDragMultiplier": 10,
    "torqueFactor": 1, "torqueDamping": 0.5, "boundaryFriction": 0.8, "rollingContactRadiusMultiplier": 5,
    "density": 0.1, "repulsionStrength": 200, "spawnOverlapOffset": 0.5, "splitVelocityMagnitude": 0.5,
}


def shipped_genome(pkg):
    g = pkg.CellGenome([pkg.GenomeMode(
        index=0, modeName="Mode 0", splitInterval=5.0, isInitial=True, parentMakeAdhesion=True,
        modeColor=(0.0, 0.0, 0.0, 0.0), parentSplitYaw=0.0, parentSplitPitch=0.0, childAModeIndex=0,
        childA_OrientationYaw=90.0, childA_OrientationPitch=0.0, childA_KeepAdhesion=True, childBModeIndex=0,
        childB_OrientationYaw=90.0, childB_OrientationPitch=0.0, childB_KeepAdhesion=True, adhesionRestLength=2.96,
        adhesionSpringStiffness=200.0, adhesionSpringDamping=0.0, orientationConstraintStrength=0.493,
        maxAllowedAngleDeviation=0.0, adhesionCanBreak=False, adhesionBreakForce=100.0)])
    return g


def shipped_controller(pkg, device=0, backend=None, bonds=False):
    """The scene's controller; bonds=True also attaches the CellAdhesionManager mirror (the scene's
    manager object, `Particle Simulation.unity`), so divisions create the genome's bonds."""
    ctl = pkg.ParticleSystemController(particleCount=SCENE_CONTROLLER["particleCount"], device=device, backend=backend)
    for k, v in SCENE_CONTROLLER.items():
        if k != "particleCount":
            setattr(ctl, k, float(v))
    ctl.genome = shipped_genome(pkg)
    if bonds:
        ctl.adhesionManager = pkg.CellAdhesionManager(ctl)
    return ctl
