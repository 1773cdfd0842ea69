"""Tracker front-ends (reference: boxmot/trackers/*)."""
