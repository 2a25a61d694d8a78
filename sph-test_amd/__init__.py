"""sph_test_amd — MI355X-native particle step behind the reference's controller API.

Product = libsphhip.so (HIP kernels for gfx950 + C ABI, include/sphhip.h). This package
is the host-side mirror of the reference's controller (ParticleSystemController.cs) and the
north-star SPHSim controller over that library. It has no CPU compute path: the library must
load, or every call raises.
"""
from ._abi import (ADHESION84, PARTICLE84, SPLIT92, SPH_MODEL_CONTACT, SPH_MODEL_WCSPH, SPH_SCENARIO_DAMBREAK,  # noqa: F401
                   SPH_SCENARIO_SLOSHING, SphError, SphParams, SphScenario, lib, LIB_PATH)
from .context import Context, comm_unique_id, make_scenario, scenario_params  # noqa: F401
from .adhesion_manager import AdhesionBond, BondZone, CellAdhesionManager  # noqa: F401
from .controllers import CONFIGS, ParticleIDData, ParticleSystemController, SPHSim, config_scenario  # noqa: F401
from .genome import CellGenome, GenomeMode, load_genome_asset, load_scene_controller  # noqa: F401

__all__ = ["Context", "CellAdhesionManager", "BondZone", "comm_unique_id", "SPHSim", "ParticleSystemController", "CONFIGS", "config_scenario",
           "make_scenario", "scenario_params", "ADHESION84", "PARTICLE84", "SPLIT92", "CellGenome", "GenomeMode",
           "ParticleIDData", "load_genome_asset", "load_scene_controller", "SphError", "SphParams", "SphScenario",
           "lib", "LIB_PATH"]
