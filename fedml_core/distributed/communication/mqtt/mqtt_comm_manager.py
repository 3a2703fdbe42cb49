"""Compat shim: reference import path ``fedml_core/distributed/communication/mqtt/mqtt_comm_manager.py`` -> ``neuroimagedisttraining_amd.comm.managers``."""
from neuroimagedisttraining_amd.comm.managers import MqttCommManager  # noqa: F401
