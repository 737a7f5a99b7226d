"""MI355X-native Grounding DINO (reference models/GroundingDINO/)."""
from .groundingdino import build_groundingdino  # noqa: F401
