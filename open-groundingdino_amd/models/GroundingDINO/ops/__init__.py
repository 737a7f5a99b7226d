"""Op layer: MI355X-native replacement of the reference's Deformable-DETR
extension package models/GroundingDINO/ops/ (functions/, modules/)."""
