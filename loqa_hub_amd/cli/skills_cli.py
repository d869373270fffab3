"""``skills-cli``: HTTP client for ``/api/skills`` (``cmd/skills-cli/main.go``).

    python -m loqa_hub_amd.cli.skills_cli -hub http://localhost:3000 -action list
    -action list|info|load|unload|enable|disable|reload  -skill ID  -path DIR
    -format table|json  -v

Output strings and exit codes follow the reference (:95-166, :175-399). The
reference decodes ``config.timeout`` as a string although the API sends Go
nanoseconds; both forms are accepted here.
"""
from __future__ import annotations

import argparse
import json
import sys
import urllib.error
import urllib.request
from datetime import datetime

from ..utils.security import sanitize_log_input as san

DEFAULT_HUB_URL = "http://localhost:3000"
ACTIONS = ("list", "load", "unload", "enable", "disable", "reload", "info")


class CLIError(Exception):
    pass


def _req(method: str, url: str, body: dict | None = None) -> tuple[int, bytes]:
    data = json.dumps(body).encode() if body is not None else None
    r = urllib.request.Request(url, data=data, method=method,
                               headers={"Content-Type": "application/json"} if data else {})
    try:
        with urllib.request.urlopen(r, timeout=30) as resp:
            return resp.status, resp.read()
    except urllib.error.HTTPError as e:
        return e.code, e.read()
    except (urllib.error.URLError, OSError) as e:
        raise CLIError(f"failed to connect to hub: {e}") from e


def _fmt_time(s: str | None, fmt: str) -> str:
    if not s or s.startswith("0001-01-01"):
        return ""
    try:
        return datetime.fromisoformat(s.replace("Z", "+00:00")[:26] + (
            "+00:00" if s.endswith("Z") else "")).strftime(fmt)
    except ValueError:
        return s


def _fmt_bool(b: bool) -> str:
    return "✓" if b else "✗"


def _fmt_timeout(v) -> str:
    if isinstance(v, (int, float)):
        from ..config import format_go_duration
        return format_go_duration(v / 1e9)
    return str(v)


class SkillCLI:
    def __init__(self, hub_url: str = DEFAULT_HUB_URL, verbose: bool = False, fmt: str = "table",
                 out=None):
        self.hub, self.verbose, self.fmt = hub_url.rstrip("/"), verbose, fmt
        self.out = out or sys.stdout

    def p(self, s: str = "") -> None:
        self.out.write(s + "\n")

    def list_skills(self) -> None:
        st, body = _req("GET", self.hub + "/api/skills")
        if st != 200:
            raise CLIError(f"API returned status {st}")
        try:
            res = json.loads(body)
        except ValueError as e:
            raise CLIError(f"failed to parse response: {e}") from e
        skills = res.get("skills") or []
        if self.fmt == "json":
            self.p(json.dumps(skills, indent=2))
            return
        rows = [("ID", "NAME", "VERSION", "STATUS", "ENABLED", "ERRORS", "LAST USED"),
                ("---", "----", "-------", "------", "-------", "------", "---------")]
        for s in skills:
            m, c, stt = s.get("manifest", {}), s.get("config", {}), s.get("status", {})
            rows.append((san(m.get("id", "")), san(m.get("name", "")), san(m.get("version", "")),
                         stt.get("state", ""), _fmt_bool(bool(c.get("enabled"))),
                         str(s.get("error_count", 0)),
                         _fmt_time(s.get("last_used"), "%Y-%m-%d %H:%M") or "never"))
        widths = [max(len(r[i]) for r in rows) for i in range(len(rows[0]))]
        for r in rows:
            self.p("  ".join(v.ljust(w) for v, w in zip(r, widths)).rstrip())
        self.p(f"\nTotal: {res.get('count', len(skills))} skills")

    def get_skill(self, sid: str) -> None:
        st, body = _req("GET", f"{self.hub}/api/skills/{sid}")
        if st == 404:
            raise CLIError(f"skill {sid} not found")
        if st != 200:
            raise CLIError(f"API returned status {st}")
        s = json.loads(body)
        if self.fmt == "json":
            self.p(json.dumps(s, indent=2))
            return
        m, c, stt = s.get("manifest", {}), s.get("config", {}), s.get("status", {})
        self.p("Skill Information:")
        for label, key in (("ID", "id"), ("Name", "name"), ("Version", "version"),
                           ("Description", "description"), ("Author", "author"),
                           ("License", "license")):
            self.p(f"  {label + ':':<13}{san(m.get(key, ''))}")
        self.p("\nStatus:")
        self.p(f"  State:       {stt.get('state', '')}")
        self.p(f"  Healthy:     {_fmt_bool(bool(stt.get('healthy')))}")
        self.p(f"  Enabled:     {_fmt_bool(bool(c.get('enabled')))}")
        self.p(f"  Loaded At:   {_fmt_time(s.get('loaded_at'), '%Y-%m-%d %H:%M:%S')}")
        if s.get("last_used"):
            self.p(f"  Last Used:   {_fmt_time(s.get('last_used'), '%Y-%m-%d %H:%M:%S')}")
        self.p(f"  Usage Count: {stt.get('usage_count', 0)}")
        self.p(f"  Error Count: {s.get('error_count', 0)}")
        if s.get("last_error"):
            self.p(f"  Last Error:  {san(s['last_error'])}")
        self.p("\nConfiguration:")
        self.p(f"  Timeout:     {_fmt_timeout(c.get('timeout', ''))}")
        self.p(f"  Max Retries: {c.get('max_retries', 0)}")
        self.p(f"  Plugin Path: {san(s.get('plugin_path', ''))}")
        if c.get("config"):
            self.p("\nCustom Config:")
            for k, v in c["config"].items():
                self.p(f"  {san(k)}: {v}")

    def load_skill(self, path: str) -> None:
        st, body = _req("POST", self.hub + "/api/skills", {"skill_path": path})
        if st == 409:
            raise CLIError("skill already loaded")
        if st != 201:
            raise CLIError(f"API returned status {st}: {body.decode(errors='replace')}")
        self.p(f"Skill loaded successfully from {san(path)}")

    def unload_skill(self, sid: str) -> None:
        st, _ = _req("DELETE", f"{self.hub}/api/skills/{sid}")
        if st == 404:
            raise CLIError(f"skill {sid} not found")
        if st != 200:
            raise CLIError(f"API returned status {st}")
        self.p(f"Skill {san(sid)} unloaded successfully")

    def skill_action(self, sid: str, action: str) -> None:
        st, body = _req("POST", f"{self.hub}/api/skills/{sid}/{action}")
        if st == 404:
            raise CLIError(f"skill {sid} not found")
        if st != 200:
            raise CLIError(f"API returned status {st}: {body.decode(errors='replace')}")
        self.p(f"Skill {san(sid)} {action}d successfully")


def main(argv=None, out=None, err=None) -> int:
    err = err or sys.stderr
    ap = argparse.ArgumentParser(prog="skills-cli", prefix_chars="-")
    ap.add_argument("-hub", "--hub", default=DEFAULT_HUB_URL, help="URL of the Loqa hub")
    ap.add_argument("-action", "--action", default="list",
                    help="Action to perform: list, load, unload, enable, disable, reload, info")
    ap.add_argument("-skill", "--skill", default="", help="Skill ID for actions")
    ap.add_argument("-path", "--path", default="", help="Path to skill directory for load action")
    ap.add_argument("-v", action="store_true", help="Verbose output")
    ap.add_argument("-format", "--format", default="table", help="Output format: table, json")
    a = ap.parse_args(argv)
    cli = SkillCLI(a.hub, a.v, a.format, out)
    try:
        if a.action == "list":
            cli.list_skills()
        elif a.action == "load":
            if not a.path:
                err.write("Error: skill path required for load action\n")
                return 1
            cli.load_skill(a.path)
        elif a.action in ACTIONS:
            if not a.skill:
                err.write(f"Error: skill ID required for {a.action} action\n")
                return 1
            if a.action == "info":
                cli.get_skill(a.skill)
            elif a.action == "unload":
                cli.unload_skill(a.skill)
            else:
                cli.skill_action(a.skill, a.action)
        else:
            err.write(f"Error: unknown action {a.action}\n")
            err.write("Valid actions: list, load, unload, enable, disable, reload, info\n")
            return 1
    except CLIError as e:
        err.write(f"Error: {e}\n")
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
