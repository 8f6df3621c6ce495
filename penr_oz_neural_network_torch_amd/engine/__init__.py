"""Device-resident fused training engine (flat params, fused optimizer, explicit fwd/bwd schedule)."""
