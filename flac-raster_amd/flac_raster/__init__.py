"""flac_raster -- MI355X-native (gfx950 HIP) FLAC encoder for rasters, API-compatible with
yharby/flac-raster's ``flac_raster`` package on the encode path."""
__version__ = "0.2.0"
