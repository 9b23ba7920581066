"""mqr -- MI355X-native TSDF fusion path for Quest depth captures."""
__version__ = "0.1.0"
