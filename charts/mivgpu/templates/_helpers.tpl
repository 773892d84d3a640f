{{- define "mivgpu.name" -}}
{{- default .Chart.Name .Values.nameOverride | trunc 63 | trimSuffix "-" -}}
{{- end -}}

{{- define "mivgpu.fullname" -}}
{{- if .Values.fullnameOverride -}}
{{- .Values.fullnameOverride | trunc 63 | trimSuffix "-" -}}
{{- else -}}
{{- printf "%s-%s" .Release.Name (include "mivgpu.name" .) | trunc 63 | trimSuffix "-" -}}
{{- end -}}
{{- end -}}

{{- define "mivgpu.namespace" -}}
{{- default .Release.Namespace .Values.namespaceOverride -}}
{{- end -}}

{{- define "mivgpu.scheduler" -}}{{ include "mivgpu.fullname" . }}-scheduler{{- end -}}
{{- define "mivgpu.devicePlugin" -}}{{ include "mivgpu.fullname" . }}-device-plugin{{- end -}}

{{- define "mivgpu.labels" -}}
app.kubernetes.io/name: {{ include "mivgpu.name" . }}
app.kubernetes.io/instance: {{ .Release.Name }}
app.kubernetes.io/version: {{ .Chart.AppVersion | quote }}
app.kubernetes.io/managed-by: {{ .Release.Service }}
helm.sh/chart: {{ printf "%s-%s" .Chart.Name .Chart.Version }}
{{- end -}}

{{- define "mivgpu.image" -}}
{{- $tag := default .Chart.AppVersion .Values.image.tag -}}
{{- if .Values.image.registry -}}
{{ printf "%s/%s:%s" .Values.image.registry .Values.image.repository $tag }}
{{- else -}}
{{ printf "%s:%s" .Values.image.repository $tag }}
{{- end -}}
{{- end -}}

{{- define "mivgpu.managedResources" -}}
- name: {{ .Values.resources.count }}
  ignoredByScheduler: true
- name: {{ .Values.resources.memory }}
  ignoredByScheduler: true
- name: {{ .Values.resources.memoryPercentage }}
  ignoredByScheduler: true
- name: {{ .Values.resources.cores }}
  ignoredByScheduler: true
- name: {{ .Values.resources.priority }}
  ignoredByScheduler: true
{{- end -}}
