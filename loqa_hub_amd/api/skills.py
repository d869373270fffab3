"""``/api/skills`` admin REST surface (``internal/api/skills.go``).

GET    /api/skills                      {skills: [...SkillInfo], count}
POST   /api/skills                      {skill_path} -> 201 {message, path}; 409 if loaded
GET    /api/skills/{id}                 SkillInfo | 404
DELETE /api/skills/{id}                 unload
PUT    /api/skills/{id}                 {config} -> update
POST   /api/skills/{id}/{enable|disable|reload}

Errors use the reference's JSON shape ``{"error": true, "message": ...}``
(:372-385); ids are validated with ``validate_skill_id`` (:35-90). The reference
never routes this handler; the hub server here does. Deliberate
fix: PUT actually applies the config (reference :320-353 mutates a copy and
persists nothing).
"""
from __future__ import annotations

import json

from aiohttp import web

from ..skills.manager import SkillAlreadyLoaded, SkillManager, SkillNotFound
from ..utils import gojson
from ..utils.security import InvalidSkillID, sanitize_log_input, validate_skill_id

VALID_ACTIONS = ("enable", "disable", "reload")


def write_json(status: int, data) -> web.Response:
    return web.Response(status=status, text=gojson.dumps(data) + "\n",
                        content_type="application/json")


def write_error(status: int, message: str) -> web.Response:
    return write_json(status, {"error": True, "message": message})


def extract_skill_id(path: str) -> str:
    parts = path.strip("/").split("/")
    return parts[2] if len(parts) >= 3 and parts[0] == "api" and parts[1] == "skills" else ""


def extract_skill_id_and_action(path: str) -> tuple[str, str]:
    parts = path.strip("/").split("/")
    if len(parts) >= 4 and parts[0] == "api" and parts[1] == "skills":
        return parts[2], parts[3]
    return "", ""


class SkillsHandler:
    def __init__(self, manager: SkillManager):
        self.manager = manager

    def routes(self) -> list[web.RouteDef]:
        return [web.route("*", "/api/skills", self.handle_skills),
                web.route("*", "/api/skills/{tail:.*}", self.handle_tail)]

    async def handle_skills(self, req: web.Request) -> web.Response:
        if req.method == "GET":
            return self.list_skills()
        if req.method == "POST":
            return await self.load_skill(req)
        return write_error(405, "method not allowed")

    async def handle_tail(self, req: web.Request) -> web.Response:
        parts = [p for p in req.match_info.get("tail", "").strip("/").split("/")]
        if len(parts) >= 2:
            return await self.handle_skill_action(req)
        return await self.handle_skill_by_id(req)

    async def handle_skill_by_id(self, req: web.Request) -> web.Response:
        sid = extract_skill_id(req.path)
        try:
            validate_skill_id(sid)
        except InvalidSkillID:
            return write_error(400, "invalid skill ID")
        if req.method == "GET":
            return self.get_skill(sid)
        if req.method == "DELETE":
            return await self._do(self.manager.unload_skill, sid, "unload",
                                  "skill unloaded successfully")
        if req.method == "PUT":
            return await self.update_skill(req, sid)
        return write_error(405, "method not allowed")

    async def handle_skill_action(self, req: web.Request) -> web.Response:
        if req.method != "POST":
            return write_error(405, "method not allowed")
        sid, action = extract_skill_id_and_action(req.path)
        try:
            validate_skill_id(sid)
        except InvalidSkillID:
            return write_error(400, "invalid skill ID or action")
        if action not in VALID_ACTIONS:
            return write_error(400, "invalid skill ID or action")
        if action == "enable":
            return await self._do(self.manager.enable_skill, sid, "enable",
                                  "skill enabled successfully")
        if action == "disable":
            return await self._do(self.manager.disable_skill, sid, "disable",
                                  "skill disabled successfully")
        return await self.reload_skill(sid)

    def list_skills(self) -> web.Response:
        infos = self.manager.list_skills()
        return write_json(200, {"skills": [i.to_go() for i in infos], "count": len(infos)})

    def get_skill(self, sid: str) -> web.Response:
        try:
            return write_json(200, self.manager.get_skill(sid).to_go())
        except SkillNotFound:
            return write_error(404, "skill not found")
        except Exception:  # noqa: BLE001
            return write_error(500, "failed to get skill")

    async def load_skill(self, req: web.Request) -> web.Response:
        try:
            body = json.loads(await req.read())
            path = body.get("skill_path", "") if isinstance(body, dict) else None
            if path is None or not isinstance(path, str):
                raise ValueError
        except ValueError:
            return write_error(400, "invalid request body")
        if path == "":
            return write_error(400, "skill_path is required")
        try:
            await self.manager.load_skill(path)
        except SkillAlreadyLoaded:
            return write_error(409, "skill already loaded")
        except Exception as e:  # noqa: BLE001
            return write_error(500, "failed to load skill: " + str(e))
        return write_json(201, {"message": "skill loaded successfully", "path": path})

    async def _do(self, fn, sid: str, verb: str, ok_msg: str) -> web.Response:
        try:
            await fn(sid)
        except SkillNotFound:
            return write_error(404, "skill not found")
        except Exception:  # noqa: BLE001
            return write_error(500, f"failed to {verb} skill")
        return write_json(200, {"message": ok_msg, "skill": sid})

    async def reload_skill(self, sid: str) -> web.Response:
        try:
            self.manager.get_skill(sid)
        except SkillNotFound:
            return write_error(404, "skill not found")
        try:
            await self.manager.reload_skill(sid)
        except SkillNotFound:
            return write_error(500, "failed to unload skill")
        except Exception as e:  # noqa: BLE001
            return write_error(500, "failed to reload skill: " + sanitize_log_input(str(e)))
        return write_json(200, {"message": "skill reloaded successfully", "skill": sid})

    async def update_skill(self, req: web.Request, sid: str) -> web.Response:
        try:
            body = json.loads(await req.read())
            if not isinstance(body, dict):
                raise ValueError
        except ValueError:
            return write_error(400, "invalid request body")
        try:
            self.manager.get_skill(sid)
        except SkillNotFound:
            return write_error(404, "skill not found")
        cfg = body.get("config")
        if isinstance(cfg, dict):
            try:
                await self.manager.update_skill_config(sid, cfg)
            except Exception:  # noqa: BLE001
                return write_error(500, "failed to update skill")
        return write_json(200, {"message": "skill configuration updated successfully",
                                "skill": sid})
