"""Post-processing of tracker results (boxmot/postprocessing/): gsi.py (GSI), mot.py (MOT rows)."""
