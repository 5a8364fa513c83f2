"""istio_amd -- MI355X-native batched policy engine for Istio Mixer's Check predicate path."""
