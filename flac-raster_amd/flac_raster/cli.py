"""``flac-raster`` command line (commands and options of the reference's ``cli.py``).

convert / info / extract / query / compare keep the reference's arguments (``cli.py:51-444``);
``convert`` adds ``--devices`` (comma-separated GPU ids) for the multi-GPU tile split.  Remote
inputs (http/s3/az/gs) are out of scope for this build and are rejected with a clear message.
"""

from __future__ import annotations

import json
import logging
import tempfile
from pathlib import Path
from typing import List, Optional

import typer
from rich.console import Console
from rich.logging import RichHandler
from rich.table import Table

from .compare import compare_tiffs, display_comparison_table
from .converter import RasterFLACConverter

app = typer.Typer(name="flac-raster",
                  help="Convert GeoTIFF raster data to/from FLAC format with spatial streaming support (MI355X).",
                  add_completion=False, no_args_is_help=True)
console = Console()
logging.basicConfig(level=logging.INFO, format="%(message)s", datefmt="[%X]",
                    handlers=[RichHandler(console=console, rich_tracebacks=True)])
logger = logging.getLogger("flac_raster")

_REMOTE = ("http://", "https://", "s3://", "az://", "gs://")


def _local(path: str) -> Path:
    if path.startswith(_REMOTE):
        raise typer.BadParameter("remote URLs are not supported by this build; download the file first")
    return Path(path)


def _devices(spec: Optional[str]) -> Optional[List[int]]:
    if not spec:
        return None
    return [int(x) for x in spec.split(",") if x.strip()]


@app.command()
def convert(
    input_file: str = typer.Argument(..., help="Input file (TIFF or FLAC)"),
    output_file: Optional[Path] = typer.Option(None, "--output", "-o", help="Output file path"),
    compression_level: int = typer.Option(5, "--compression", "-c", min=0, max=8, help="FLAC compression level"),
    spatial: bool = typer.Option(False, "--spatial", "-s", help="Enable spatial tiling for streaming"),
    tile_size: int = typer.Option(512, "--tile-size", "-t", help="Tile size in pixels (default: 512)"),
    streaming: bool = typer.Option(False, "--streaming", help="Streaming format (each tile is a complete FLAC)"),
    force: bool = typer.Option(False, "--force", "-f", help="Overwrite existing output file"),
    verbose: bool = typer.Option(False, "--verbose", "-v", help="Enable verbose logging"),
    devices: Optional[str] = typer.Option(None, "--devices", help="GPU ids to split tiles over, e.g. 0,1,2,3"),
):
    """Convert between TIFF and FLAC formats."""
    if verbose:
        logging.getLogger("flac_raster").setLevel(logging.DEBUG)
    try:
        src = _local(input_file)
        if not src.exists():
            console.print(f"[red]Error: Input file does not exist: {src}[/red]")
            raise typer.Exit(1)
        suffix = src.suffix.lower()
        if suffix in (".tif", ".tiff"):
            direction, default_suffix = "tiff_to_flac", ".flac"
        elif suffix == ".flac":
            direction, default_suffix = "flac_to_tiff", ".tif"
        else:
            console.print(f"[red]Error: Unsupported format: {suffix}[/red]")
            raise typer.Exit(1)
        if output_file is None:
            output_file = (src.with_name(f"{src.stem}_streaming{default_suffix}") if streaming
                           else src.with_suffix(default_suffix))
        if output_file.exists() and not force:
            console.print(f"[red]Error: Output exists: {output_file}[/red]")
            raise typer.Exit(1)
        devs = _devices(devices)
        if streaming and direction == "tiff_to_flac":
            from .streaming import create_streaming_flac

            idx = create_streaming_flac(src, output_file, tile_size, compression_level, devs)
            console.print(f"[green]Created streaming FLAC: {output_file} ({len(idx['frames'])} tiles, "
                          f"{output_file.stat().st_size / 1024 / 1024:.2f} MB)[/green]")
            return
        conv = RasterFLACConverter(devices=devs)
        if direction == "tiff_to_flac":
            res = conv.tiff_to_flac(src, output_file, compression_level, spatial, tile_size)
            if spatial and res:
                console.print(f"[green]Created {len(res.frames)} spatial tiles[/green]")
        else:
            conv.flac_to_tiff(src, output_file)
    except typer.Exit:
        raise
    except Exception as e:
        logger.exception("Conversion failed")
        console.print(f"[red]Error: {e}[/red]")
        raise typer.Exit(1)


@app.command()
def info(file_path: str = typer.Argument(..., help="File to inspect")):
    """Display information about a FLAC or TIFF file."""
    try:
        p = _local(file_path)
        if not p.exists():
            console.print(f"[red]Error: File not found: {p}[/red]")
            raise typer.Exit(1)
        s = p.suffix.lower()
        if s in (".tif", ".tiff"):
            _show_tiff_info(p)
        elif s == ".flac":
            _show_flac_info(p)
        else:
            console.print(f"[red]Unsupported format: {s}[/red]")
            raise typer.Exit(1)
    except typer.Exit:
        raise
    except Exception as e:
        logger.exception("Info failed")
        console.print(f"[red]Error: {e}[/red]")
        raise typer.Exit(1)


@app.command()
def extract(
    flac_file: str = typer.Argument(..., help="Streaming FLAC file"),
    output: Path = typer.Option(..., "--output", "-o", help="Output TIFF file path"),
    bbox: Optional[str] = typer.Option(None, "--bbox", "-b", help="Bounding box: 'xmin,ymin,xmax,ymax'"),
    tile_id: Optional[int] = typer.Option(None, "--tile-id", help="Extract specific tile by ID"),
    center: bool = typer.Option(False, "--center", help="Extract center tile"),
    last: bool = typer.Option(False, "--last", help="Extract last tile"),
):
    """Extract one tile of a streaming FLAC file to GeoTIFF."""
    from .streaming import open_streaming, read_tile_bytes, select_frame

    try:
        path = _local(flac_file)
        sf = open_streaming(path)
        frames = sf.index["frames"]
        console.print(f"[green]Found {len(frames)} tiles[/green]")
        coords = [float(x.strip()) for x in bbox.split(",")] if bbox else None
        fr = select_frame(frames, tile_id=tile_id, bbox=coords, center=center, last=last)
        data = read_tile_bytes(path, fr, sf.header_size)
        with tempfile.NamedTemporaryFile(suffix=".flac", delete=False) as tmp:
            tmp.write(data)
            tmp_path = Path(tmp.name)
        try:
            RasterFLACConverter().flac_to_tiff(tmp_path, output)
        finally:
            tmp_path.unlink()
        total = sum(f["byte_size"] for f in frames)
        console.print(f"[green]Saved to: {output}[/green]")
        console.print(f"[blue]Bandwidth: {fr['byte_size'] / 1024:.1f} KB "
                      f"(saved {(1 - fr['byte_size'] / total) * 100:.1f}%)[/blue]")
    except typer.Exit:
        raise
    except Exception as e:
        logger.exception("Extraction failed")
        console.print(f"[red]Error: {e}[/red]")
        raise typer.Exit(1)


@app.command()
def query(
    flac_file: str = typer.Argument(..., help="Spatial FLAC file"),
    bbox: str = typer.Option(..., "--bbox", "-b", help="Bounding box: 'xmin,ymin,xmax,ymax'"),
    output: Optional[Path] = typer.Option(None, "--output", "-o", help="Save byte ranges to JSON file"),
):
    """Byte ranges of the tiles of a spatial FLAC file that intersect a bbox."""
    from .spatial_encoder import SpatialFLACStreamer

    try:
        coords = tuple(float(x.strip()) for x in bbox.split(","))
        if len(coords) != 4:
            console.print("[red]Bbox must have 4 coordinates[/red]")
            raise typer.Exit(1)
        ranges = SpatialFLACStreamer(_local(flac_file)).get_byte_ranges_for_bbox(coords)
        total = sum(e - s + 1 for s, e in ranges)
        t = Table(title=f"Byte Ranges for bbox {bbox}")
        for name, style in (("#", "cyan"), ("Start", "green"), ("End", "yellow"), ("Size", "blue"),
                            ("Range Header", "magenta")):
            t.add_column(name, style=style)
        for i, (s, e) in enumerate(ranges, 1):
            t.add_row(str(i), f"{s:,}", f"{e:,}", f"{e - s + 1:,}", f"bytes={s}-{e}")
        console.print(t)
        console.print(f"[bold]Total: {total:,} bytes ({len(ranges)} ranges)[/bold]")
        if output:
            output.write_text(json.dumps({"bbox": list(coords), "ranges": [{"start": s, "end": e} for s, e in ranges],
                                          "total_bytes": total}, indent=2))
    except typer.Exit:
        raise
    except Exception as e:
        logger.exception("Query failed")
        console.print(f"[red]Error: {e}[/red]")
        raise typer.Exit(1)


@app.command()
def compare(
    file1: Path = typer.Argument(..., help="First TIFF file"),
    file2: Path = typer.Argument(..., help="Second TIFF file"),
    show_bands: bool = typer.Option(True, "--show-bands/--no-bands", help="Show per-band statistics"),
    export_json: Optional[Path] = typer.Option(None, "--export", "-e", help="Export comparison to JSON"),
):
    """Compare two TIFF files."""
    for f in (file1, file2):
        if not f.exists():
            console.print(f"[red]File not found: {f}[/red]")
            raise typer.Exit(1)
        if f.suffix.lower() not in (".tif", ".tiff"):
            console.print(f"[red]Not a TIFF file: {f}[/red]")
            raise typer.Exit(1)
    res = compare_tiffs(file1, file2, show_bands)
    display_comparison_table(res)
    if export_json:
        export_json.write_text(json.dumps(res, indent=2, default=list))


def _show_tiff_info(path: Path):
    from .tiff import GeoTIFF

    info = GeoTIFF(path).info
    from .geo import Affine, bounds

    l, b, r, t = bounds(Affine(*info.transform), info.width, info.height)
    tab = Table(title=f"TIFF: {path.name}")
    tab.add_column("Property", style="cyan")
    tab.add_column("Value", style="green")
    tab.add_row("Dimensions", f"{info.width} x {info.height}")
    tab.add_row("Bands", str(info.count))
    tab.add_row("Data Type", str(info.dtype))
    tab.add_row("CRS", str(info.crs))
    tab.add_row("Bounds", f"({l:.6f}, {b:.6f}, {r:.6f}, {t:.6f})")
    tab.add_row("File Size", f"{path.stat().st_size / 1024 / 1024:.2f} MB")
    console.print(tab)


def _show_flac_info(path: Path):
    from . import flac_meta

    f = flac_meta.FLACFile(path)
    tab = Table(title=f"FLAC: {path.name}")
    tab.add_column("Property", style="cyan")
    tab.add_column("Value", style="green")
    tab.add_row("Sample Rate", f"{f.sample_rate} Hz")
    tab.add_row("Channels", str(f.channels))
    tab.add_row("Bits per Sample", str(f.bits_per_sample))
    tab.add_row("File Size", f"{path.stat().st_size / 1024 / 1024:.2f} MB")
    console.print(tab)
    if "GEOSPATIAL_CRS" in f:
        g = Table(title="Geospatial Metadata")
        g.add_column("Property", style="cyan")
        g.add_column("Value", style="green")
        get = lambda k, d="?": f.get(k, [d])[0]  # noqa: E731
        g.add_row("Dimensions", f"{get('GEOSPATIAL_WIDTH')} x {get('GEOSPATIAL_HEIGHT')}")
        g.add_row("Bands", get("GEOSPATIAL_COUNT"))
        g.add_row("Original Type", get("GEOSPATIAL_DTYPE"))
        g.add_row("CRS", get("GEOSPATIAL_CRS"))
        g.add_row("Data Range", f"[{get('GEOSPATIAL_DATA_MIN')}, {get('GEOSPATIAL_DATA_MAX')}]")
        g.add_row("Spatial Tiling", get("GEOSPATIAL_SPATIAL_TILING", "false"))
        console.print(g)


def main():
    app()


if __name__ == "__main__":
    main()
