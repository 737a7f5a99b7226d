"""MI355X-native Grounding DINO (reference models/GroundingDINO/)."""
