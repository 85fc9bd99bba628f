"""Hyper-parameter advisors (GP-EI Bayesian optimisation, random search) and their REST service."""
from .advisor import Advisor, BaseAdvisor, GpAdvisor, RandomAdvisor, make_advisor  # noqa: F401
from ..constants import AdvisorType  # noqa: F401
