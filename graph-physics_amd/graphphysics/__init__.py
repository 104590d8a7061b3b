"""graphphysics (MI355X-native MGN hot path) — drop-in for the reference package's MeshGraphNet
training path (cviviers/graph-physics). See DESIGN.md at the repository root."""
__version__ = "0.1.0"
