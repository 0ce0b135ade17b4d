"""deap_amd — MI355X-native population evaluator for DEAP-style genetic programming.

The package mirrors the DEAP API surface the GP hot path touches
(``base``, ``creator``, ``gp``, ``tools``, ``algorithms``) and adds the GPU
evaluator (:mod:`deap_amd.evaluator`) that replaces the per-individual
``gp.compile`` + Python per-case loop behind ``toolbox.register("map"/"evaluate")``.
"""
__version__ = "0.1.0"
