"""Drop-in mirror of the reference's ``spotlight`` package surface used by the
MF/NCF training path (spotlight/ in the reference): the same module names,
classes and functions, with training routed through librg_hip.so."""
