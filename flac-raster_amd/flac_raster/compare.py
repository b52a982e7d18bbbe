"""TIFF comparison report (``compare.py`` of the reference: ``compare_tiffs`` +
``display_comparison_table``), on the in-package GeoTIFF reader."""

from __future__ import annotations

import logging
from pathlib import Path

import numpy as np
from rich.console import Console
from rich.table import Table

from .tiff import GeoTIFF

console = Console()
logger = logging.getLogger("flac_raster.compare")


def compare_tiffs(file1_path: Path, file2_path: Path, show_bands: bool = True) -> dict:
    p1, p2 = Path(file1_path), Path(file2_path)
    g1, g2 = GeoTIFF(p1), GeoTIFF(p2)
    d1, d2 = g1.read(), g2.read()
    r = {
        "file1": p1.name, "file2": p2.name,
        "shape_match": d1.shape == d2.shape,
        "dtype_match": d1.dtype == d2.dtype,
        "crs_match": g1.info.crs == g2.info.crs,
        "file1_shape": d1.shape, "file2_shape": d2.shape,
        "file1_dtype": str(d1.dtype), "file2_dtype": str(d2.dtype),
        "file1_crs": str(g1.info.crs), "file2_crs": str(g2.info.crs),
    }
    if r["shape_match"]:
        diff = np.abs(d1 - d2)  # same (possibly wrapping) arithmetic as the reference
        r["arrays_equal"] = bool(np.array_equal(d1, d2))
        r["max_difference"] = float(np.max(diff))
        r["mean_difference"] = float(np.mean(diff))
        r["rmse"] = float(np.sqrt(np.mean((d1 - d2) ** 2)))
        r["file1_min"], r["file1_max"] = float(np.min(d1)), float(np.max(d1))
        r["file2_min"], r["file2_max"] = float(np.min(d2)), float(np.max(d2))
        if show_bands and d1.ndim == 3:
            r["bands"] = [{
                "band": i + 1,
                "equal": bool(np.array_equal(d1[i], d2[i])),
                "max_diff": float(np.max(np.abs(d1[i] - d2[i]))),
                "mean_diff": float(np.mean(np.abs(d1[i] - d2[i]))),
                "file1_range": [float(d1[i].min()), float(d1[i].max())],
                "file2_range": [float(d2[i].min()), float(d2[i].max())],
            } for i in range(d1.shape[0])]
    return r


def display_comparison_table(results: dict):
    t = Table(title="TIFF Comparison Results", show_header=True)
    t.add_column("Property", style="cyan")
    t.add_column(results["file1"], style="green")
    t.add_column(results["file2"], style="yellow")
    t.add_column("Match", style="bold")
    yn = lambda b: "YES" if b else "NO"  # noqa: E731
    t.add_row("Shape", str(results["file1_shape"]), str(results["file2_shape"]), yn(results["shape_match"]))
    t.add_row("Data Type", results["file1_dtype"], results["file2_dtype"], yn(results["dtype_match"]))
    t.add_row("CRS", results["file1_crs"], results["file2_crs"], yn(results["crs_match"]))
    console.print(t)
    if not results.get("shape_match"):
        console.print("[red]Cannot compute detailed statistics - shapes don't match![/red]")
        return
    s = Table(title="Statistical Comparison", show_header=True)
    s.add_column("Metric", style="cyan")
    s.add_column("Value", style="bold")
    s.add_row("Arrays Equal", yn(results["arrays_equal"]))
    s.add_row("Max Difference", f"{results['max_difference']:.6f}")
    s.add_row("Mean Difference", f"{results['mean_difference']:.6f}")
    s.add_row("RMSE", f"{results['rmse']:.6f}")
    console.print(s)
    rg = Table(title="Data Ranges", show_header=True)
    rg.add_column("File", style="cyan")
    rg.add_column("Min", style="blue")
    rg.add_column("Max", style="red")
    rg.add_row(results["file1"], f"{results['file1_min']:.2f}", f"{results['file1_max']:.2f}")
    rg.add_row(results["file2"], f"{results['file2_min']:.2f}", f"{results['file2_max']:.2f}")
    console.print(rg)
    if "bands" in results:
        b = Table(title="Per-Band Statistics", show_header=True)
        for name, style in (("Band", "cyan"), ("Equal", "bold"), ("Max Diff", "yellow"), ("Mean Diff", "yellow"),
                            (f"{results['file1']} Range", "green"), (f"{results['file2']} Range", "blue")):
            b.add_column(name, style=style)
        for x in results["bands"]:
            b.add_row(str(x["band"]), yn(x["equal"]), f"{x['max_diff']:.3f}", f"{x['mean_diff']:.6f}",
                      f"[{x['file1_range'][0]:.1f}, {x['file1_range'][1]:.1f}]",
                      f"[{x['file2_range'][0]:.1f}, {x['file2_range'][1]:.1f}]")
        console.print(b)
